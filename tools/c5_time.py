"""Times BASELINE configs[4] (10k-sphere scene_build_complex scene, 1920x1080)
on one GPU: SPP samples per launch (default 1), HIP events; prints rays/s."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402

W, H = 1920, 1080
SPP = int(os.environ.get("SPP", "1"))
dev = torch.device("cuda", 0)
spheres, n, cam = rtamd.scenes.complex10k()
rtamd.scenes.update_camera(cam, W, H)
sc = rtamd.SmallptScene(spheres, n)
seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
seeds = torch.empty_like(seeds0)
col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
px = torch.zeros(W * H, dtype=torch.int32, device=dev)
cnt = torch.zeros(20, dtype=torch.int64, device=dev)   # [4..7]: RT_BVH_STATS builds
st = torch.cuda.current_stream(dev)
L = rtamd.lib()


R0, R1 = 0, H
if os.environ.get("BAND"):                          # BAND=k/N: row band k of N (per-GPU work at N GPUs)
    from rtamd import dist as rdist
    k, N = (int(v) for v in os.environ["BAND"].split("/"))
    R0, R1 = rdist.row_band(k, N, H)


GROUP = os.environ.get("GROUP")                    # GROUP=k/N: interleaved 8-row groups of rank k of N


MODE = rtamd.SPT_COUNT_RAYS if os.environ.get("COUNTED") == "rays" else 0


def run(c=None):
    cp = c.data_ptr() if c is not None else None
    mode = MODE if c is not None else 0
    if GROUP:
        k, N = (int(v) for v in GROUP.split("/"))
        rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                    seeds.data_ptr(), px.data_ptr(), W, H, k, N, 0, SPP, mode, cp,
                                                    st.cuda_stream))
    else:
        rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                             seeds.data_ptr(), px.data_ptr(), W, H, R0, R1, 0, SPP, mode, cp,
                                             st.cuda_stream))


stats = getattr(L, "spt_bvh_stats_read", None)   # RT_BVH_STATS builds only
bs = (C.c_ulonglong * 24)()
if stats:
    stats(bs)
run(cnt)
torch.cuda.synchronize()
rays = int(cnt[0] + cnt[1])
if stats:
    stats(bs)
    q, wq = max(bs[5], 1), max(bs[6], 1)
    print("  bvh: per query %.2f nodes, %.2f crossed leaves, %.2f sphere tests; per wave-query %.2f loop trips, "
          "%.2f leaf-block runs, %.1f lanes; node-step lane util %.3f, leaf-block lane util %.3f" % (
              bs[0] / q, bs[1] / q, bs[2] / q, bs[3] / wq, bs[4] / wq, q / wq,
              bs[0] / (64.0 * max(bs[3], 1)), bs[1] / (64.0 * max(bs[4], 1))))
    print("  queries >= 128/512/2048 nodes: %d %d %d of %d; origin outside root box: %d queries, %.1f nodes each, "
          "%d of them >= 512; shadow: %d queries, %.1f nodes each" % (
              bs[7], bs[8], bs[9], bs[5], bs[11], bs[10] / max(bs[11], 1), bs[14], bs[12], bs[13] / max(bs[12], 1)))
    print("  alpha > 1/128: %d queries, %.1f nodes each, %d >= 512; origin > 8 root radii away: %d queries, "
          "%.1f nodes each, %d >= 512" % (bs[15], bs[16] / max(bs[15], 1), bs[20], bs[17], bs[18] / max(bs[17], 1), bs[19]))
    print("  node visits in the first 64 / 256 / 1024 nodes of the ray's octant layout: %.3f %.3f %.3f" % (
        bs[21] / max(bs[0], 1), bs[22] / max(bs[0], 1), bs[23] / max(bs[0], 1)))
ts = []
COUNTED = os.environ.get("COUNTED") in ("1", "rays")   # time the counted kernel (full, or rays-only) instead
for _ in range(int(os.environ.get("WARM", "0"))):      # uncounted frames first (they teach the tile order)
    run(None)
for _ in range(int(os.environ.get("REPS", "1"))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    run(cnt if COUNTED else None)
    b.record(st)
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = float(np.median(ts))
print("c5 %dx%d rows [%d,%d) spp=%d spheres=%d%s%s: %.2f ms (median of %d, min %.2f), rays %d, %.1f Mrays/s, sphere tests %d" % (
    W, H, R0, R1, SPP, n, " counted" if COUNTED else "", " (rays only)" if MODE else "", ms, len(ts), min(ts), rays, rays / ms / 1e3, int(cnt[2])))
if int(cnt[7]):
    q = rays
    print("  per query: %.1f nodes, %.1f sphere tests; lane trips / (64 x wave trips) = %.3f" % (
        int(cnt[4]) / q, int(cnt[5]) / q, int(cnt[6]) / (64 * int(cnt[7]))))
    print("  queries with >= 128 / 512 / 2048 node visits: %d %d %d; far (leaf scan): %d" % tuple(int(v) for v in cnt[8:12]))
    print("  >= 2048: origin-root distance <25/<50/<100/<200/<400/more: %s; shadow %d; hit %d" % (
        [int(v) for v in cnt[12:18]], int(cnt[18]), int(cnt[19])))
