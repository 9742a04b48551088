"""rtamd -- host-side Python binding of the MI355X ray-trace hot path.

Thin ctypes layer over librt_hip.so (include/rt_hip.h).  The C++ drop-in
shims (csrc/shim_*.cpp) are the reference-facing host API; this module is
what the tests, bench.py and __graft_entry__ drive.

    Whitted  : whitted_render()  ~ Engine_InitRender + Engine_Render
               (raytracer3.0.06.no_rec.samp/raytracer.cpp:278-530) on the GPU
    smallpt  : SmallptFrame.render(k)  ~ k x UpdateRenderingCPU
               (smallptgpu-v1.6/smallptCPU.cpp:77-132) on the GPU, or
               tiled in row bands over several GPUs (devices=[...]);
               SmallptMulti: the device-resident multi-GPU frame (spt_multi_*)
    Queue    : queue_render()  ~ raytracer_non_kernel
               (Raytracer3.2.03/.../raytracer_non_OpenCL.c:285-449) on the GPU
"""
import ctypes as C

import numpy as np

from . import ppm, scenes
from ._lib import (Camera, Float4, Primitive, QPrimitive, RTError, Sphere, Vec3, check, device_count, lib,
                   set_device, SPT_COST_MAX, SPT_COUNT_RAYS, SPT_LIST_SET, SPT_DIRECT_LIGHTING, SPT_PATH_TRACING)

__all__ = ["Camera", "Primitive", "QPrimitive", "Float4", "Sphere", "Vec3", "RTError", "scenes", "lib", "check",
           "device_count", "set_device", "whitted_render", "queue_render", "SmallptFrame", "SmallptScene",
           "SmallptMulti",
           "SPT_PATH_TRACING", "SPT_DIRECT_LIGHTING", "SPT_COUNT_RAYS", "SPT_COST_MAX", "SPT_LIST_SET"]


def whitted_render(w, h, row_begin=20, row_end=None, prims=None, nprims=None, frame=None,
                   counters=False):
    """Render rows [row_begin,row_end) (default the reference window
    [20, h-70)) into a uint32 [h, w] frame (zero-cleared unless given).
    Returns frame, or (frame, [traced, shadow, tests, tir]) if counters."""
    if prims is None:
        prims, nprims = scenes.whitted_scene()
    if row_end is None:
        row_end = h - 70
    if frame is None:
        frame = np.zeros((h, w), dtype=np.uint32)
    assert frame.dtype == np.uint32 and frame.shape == (h, w) and frame.flags.c_contiguous
    cnt = (C.c_uint64 * 4)()
    check(lib().rtw_render(C.addressof(prims), nprims, frame.ctypes.data, w, h, row_begin,
                           row_end, C.addressof(cnt) if counters else None))
    return (frame, list(cnt)) if counters else frame


def whitted_render_ocl(w, h, prims=None, nprims=None, frame=None, counters=False):
    """The reference's OpenCL kernel semantics (raytrace_kernel of
    openCLcode.cl): rows [20, min(530, h)) of a uint32 [h, w] frame."""
    if prims is None:
        prims, nprims = scenes.whitted_scene()
    if frame is None:
        frame = np.zeros((h, w), dtype=np.uint32)
    assert frame.dtype == np.uint32 and frame.shape == (h, w) and frame.flags.c_contiguous
    cnt = (C.c_uint64 * 4)()
    check(lib().rtw_render_ocl(C.addressof(prims), nprims, frame.ctypes.data, w, h,
                               C.addressof(cnt) if counters else None))
    return (frame, list(cnt)) if counters else frame


def queue_render(w, h, prims=None, nprims=None, counters=False):
    """raytracer_non_kernel on the GPU: the uchar4 (r, g, b, 0) frame as
    uint8 [h, w, 4].  Returns frame, or (frame, [rays, shadow rays, intersect
    calls, undefined-behaviour events]) if counters."""
    if prims is None:
        prims, nprims = scenes.queue_scene()
    frame = np.zeros((h, w, 4), dtype=np.uint8)
    cnt = (C.c_uint64 * 4)()
    check(lib().rtq_render(C.addressof(prims), nprims, frame.ctypes.data, w, h,
                           C.addressof(cnt) if counters else None))
    return (frame, list(cnt)) if counters else frame


class SmallptFrame:
    """Progressive smallpt frame state: colors / seeds / pixels exactly as
    smallptGPU.cpp's AllocateBuffers lays them out, and currentSample."""

    def __init__(self, w, h, spheres=None, nspheres=None, camera=None, seed=1,
                 mode=SPT_PATH_TRACING):
        if spheres is None:
            spheres, nspheres = scenes.cornell()
        if camera is None:
            camera = scenes.cornell_camera(w, h)
        self.w, self.h = w, h
        self.spheres, self.nspheres, self.camera, self.mode = spheres, nspheres, camera, mode
        self.colors = np.zeros(3 * w * h, dtype=np.float32)
        self.seeds = scenes.seeds(w, h, seed)
        self.pixels = np.zeros(w * h, dtype=np.uint32)
        self.current_sample = 0
        self.counters = [0, 0, 0, 0]

    def render(self, nsamples=1, counters=True, devices=None):
        """nsamples successive UpdateRenderingCPU passes on the GPU.  With
        counters=False no counter buffer is passed (the kernels without the
        work counters: the ones bench.py times).  devices=[d0, d1, ...]: the
        frame tiled in row bands over those devices (spt_render_multi; a
        device may repeat)."""
        cnt = (C.c_uint64 * 4)()
        args = (C.addressof(self.spheres), self.nspheres, C.byref(self.camera), self.colors.ctypes.data,
                self.seeds.ctypes.data, self.pixels.ctypes.data, self.w, self.h, self.current_sample,
                nsamples, self.mode, C.addressof(cnt) if counters else None)
        if devices is None:
            check(lib().spt_render(*args))
        else:
            devs = (C.c_int * len(devices))(*devices)
            check(lib().spt_render_multi(*args, devs, len(devices)))
        self.current_sample += nsamples
        self.counters = [a + b for a, b in zip(self.counters, cnt)]
        return self


class SmallptScene:
    """Prepared device scene (spt_scene_create); .handle is passed to
    spt_scene_render_async.  Freed with close() / garbage collection."""

    def __init__(self, spheres, nspheres):
        self.handle = C.c_void_p()
        check(lib().spt_scene_create(C.addressof(spheres), nspheres, C.byref(self.handle)))
        self.n = nspheres

    def close(self):
        if self.handle:
            lib().spt_scene_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SmallptMulti:
    """A frame tiled in row bands over several devices (spt_multi_*): band k
    renders pixel rows [h - rows[k+1], h - rows[k]) on devices[k]; gather()
    assembles the whole frame on every band's device (one RCCL all-gather of
    the equal padded bands, or peer copies when a device repeats)."""

    def __init__(self, w, h, devices, spheres=None, nspheres=None):
        if spheres is None:
            spheres, nspheres = scenes.cornell()
        self.w, self.h, self.devices = w, h, list(devices)
        self.handle = C.c_void_p()
        devs = (C.c_int * len(self.devices))(*self.devices)
        check(lib().spt_multi_create(C.addressof(spheres), nspheres, w, h, devs, len(self.devices),
                                     C.byref(self.handle)))
        rows = (C.c_int * (len(self.devices) + 1))()
        check(lib().spt_multi_bands(self.handle, rows))
        self.rows = list(rows)

    def set_scene(self, spheres, nspheres):
        check(lib().spt_multi_set_scene(self.handle, C.addressof(spheres), nspheres))

    def upload(self, seeds, colors=None):
        check(lib().spt_multi_upload(self.handle, colors.ctypes.data if colors is not None else None,
                                     seeds.ctypes.data))

    def render(self, camera, first_sample, nsamples, mode=SPT_PATH_TRACING, counters=False):
        check(lib().spt_multi_render_async(self.handle, C.byref(camera), first_sample, nsamples, mode,
                                           int(bool(counters))))

    def gather(self):
        check(lib().spt_multi_gather_async(self.handle))

    def sync(self):
        check(lib().spt_multi_sync(self.handle))

    def download(self, colors=None, seeds=None, pixels=None):
        ptr = lambda a: a.ctypes.data if a is not None else None  # noqa: E731
        check(lib().spt_multi_download(self.handle, ptr(colors), ptr(seeds), ptr(pixels)))

    def read_frame(self, k):
        """Band k's whole device frame: (colors float32[3*w*h], pixels uint32[w*h])."""
        col = np.empty(3 * self.w * self.h, np.float32)
        px = np.empty(self.w * self.h, np.uint32)
        check(lib().spt_multi_read_frame(self.handle, k, col.ctypes.data, px.ctypes.data))
        return col, px

    def counters(self):
        out = (C.c_uint64 * 4)()
        check(lib().spt_multi_counters(self.handle, out))
        return list(out)

    def band_buffers(self, k):
        """(device, d_colors, d_seeds, d_pixels, stream) of band k."""
        dev = C.c_int()
        p = [C.c_void_p() for _ in range(4)]
        check(lib().spt_multi_band_buffers(self.handle, k, C.byref(dev), *[C.byref(x) for x in p]))
        return (dev.value,) + tuple(x.value for x in p)

    def close(self):
        if self.handle:
            lib().spt_multi_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
