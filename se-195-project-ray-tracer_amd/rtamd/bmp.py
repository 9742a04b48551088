"""24-bit BMP writer of the 3.2.x tracer: write_bmp_file
(Raytracer3.2.03/raytracer/OpenCL Raytracer/bitmap.c:8-74, bitmap.h:8-38).

Header: 'BM', BMP_HEADER {filesz, 0, 0, 54}, BMP_INFO_HEADER {40, w, h, 1,
24, 0, pixel bytes, 2835, 2835, 0, 0}; pixel rows bottom-up (:58-71), each
pixel written b, g, r (s[2], s[1], s[0]), rows padded to 4 bytes.
"""
import struct

import numpy as np


def bmp_bytes(frame):
    """frame: uint8 [h, w, 4] uchar4 (r, g, b, 0) as raytracer_non_kernel writes it."""
    frame = np.asarray(frame, dtype=np.uint8)
    h, w = frame.shape[:2]
    row = 3 * w
    pad = 0 if row % 4 == 0 else 4 - row % 4
    size = (row + pad) * h
    head = b"BM" + struct.pack("<IHHI", 14 + 40 + size, 0, 0, 14 + 40)
    info = struct.pack("<IiiHHIIiiII", 40, w, h, 1, 24, 0, size, 2835, 2835, 0, 0)
    body = np.zeros((h, row + pad), dtype=np.uint8)
    body[:, :row] = frame[::-1, :, 2::-1].reshape(h, row)
    return head + info + body.tobytes()


def write_bmp(path, frame):
    with open(path, "wb") as f:
        f.write(bmp_bytes(frame))
