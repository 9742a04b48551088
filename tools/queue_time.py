"""Times the Raytracer3.2.03 queue tracer (rtq_render_async) on one GPU:
ms per frame (HIP events, device-resident buffers) at 800x600 and 1920x1080.
    python tools/queue_time.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    prims, n = rtamd.scenes.queue_scene()
    d_prims = torch.frombuffer(bytearray(bytes(prims)[:96 * n]), dtype=torch.uint8).to(dev)
    L = rtamd.lib()
    s = torch.cuda.current_stream(dev)
    for w, h in [(800, 600), (1920, 1080)]:
        frame = torch.zeros(w * h, dtype=torch.int32, device=dev)
        run = lambda: rtamd.check(L.rtq_render_async(d_prims.data_ptr(), n, frame.data_ptr(), w, h, 0, h,  # noqa: E731
                                                     None, s.cuda_stream))
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        print("%dx%d %.4f ms/frame, device arena %.0f MB" % (w, h, e0.elapsed_time(e1) / reps,
                                                            L.rt_cached_bytes() / 1e6), flush=True)


if __name__ == "__main__":
    main()
