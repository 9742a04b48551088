"""Kernel time of each of N row bands (rtamd.dist.row_band) of the bench frame
on one GPU: the multi-GPU load balance of the row sharding."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd import dist as rdist  # noqa: E402

W, H, SPP = 1920, 1080, 64
dev = torch.device("cuda", 0)
S, n = rtamd.scenes.cornell()
cam = rtamd.scenes.cornell_camera(W, H)
sc = rtamd.SmallptScene(S, n)
seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
seeds = torch.empty_like(seeds0)
col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
px = torch.zeros(W * H, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev)
L = rtamd.lib()
for N in (2, 4, 8):
    ts = []
    for r in range(N):
        r0, r1 = rdist.row_band(r, N, H)
        best = 1e9
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                 seeds.data_ptr(), px.data_ptr(), W, H, r0, r1, 0, SPP, 0, None,
                                                 st.cuda_stream))
            b.record(st)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        ts.append(best)
    print("N=%d band ms: %s  max/mean %.3f" % (N, " ".join("%.2f" % t for t in ts), max(ts) / np.mean(ts)))
    ts = []
    for r in range(N):                     # interleaved 8-row groups (bench.py's default split)
        best = 1e9
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                        seeds.data_ptr(), px.data_ptr(), W, H, r, N, 0, SPP, 0,
                                                        None, st.cuda_stream))
            b.record(st)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b))
        ts.append(best)
    print("N=%d group ms: %s  max/mean %.3f" % (N, " ".join("%.2f" % t for t in ts), max(ts) / np.mean(ts)))
