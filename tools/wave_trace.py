"""Wave timeline of the smallpt kernel (tools-only RT_SPT_TRACE build):
per wave start/end (s_memrealtime, 100 MHz), the SIMD it ran on, and its
lanes' loop iterations.  Reports, for the full 1920x1080 frame (N=1) and one
row band of N=2/4/8, the kernel span, how busy the SIMDs were over time (the
drain tail), waves per SIMD, and the spread of per-wave work.

    tools/build_variants.sh trace -DRT_SPT_TRACE
    RT_HIP_LIB=build_ab/trace/librt_hip.so python tools/wave_trace.py [--save DIR]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd import dist as rdist  # noqa: E402

W, H, SPP = 1920, 1080, int(os.environ.get("SPP", "64"))


def run(L, sc, cam, seeds0, seeds, col, px, r0, r1, st):
    ntiles = ((W + 7) // 8) * ((r1 - r0 + 7) // 8)
    gx, gy = (ntiles + 15) // 16, 16           # blocks (upper bound), waves per block
    nw = gx * gy
    buf = torch.zeros(nw * 16, dtype=torch.int32, device=seeds.device)
    rtamd.check(L.spt_trace_set(C.c_void_p(buf.data_ptr())))
    rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                         seeds.data_ptr(), px.data_ptr(), W, H, r0, r1, 0, SPP, 0, None,
                                         st.cuda_stream))
    torch.cuda.synchronize()
    rtamd.check(L.spt_trace_set(None))
    t = buf.cpu().numpy().view(np.uint32).reshape(nw, 16).astype(np.int64)
    return t, gx, gy


def analyse(tag, t, gx, gy, save=None):
    t = t[t[:, 1] != 0]                              # waves that ran
    t0, t1, hw, xcc, iters, mx = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4], t[:, 5]
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    base = t0.min()
    s, e = (t0 - base) * 10e-6, (t1 - base) * 10e-6          # ms
    simd = ((xcc & 0xf) << 16) | (hw & 0xff30)      # XCC | SE, SH, CU, SIMD fields of HW_ID
    span = e.max()
    live = iters > 0
    u, cnt = np.unique(simd[live], return_counts=True)
    nsimd = len(u)
    # SIMD busy fraction over time: a SIMD is "busy" while >= 1 wave of it is live
    grid = np.linspace(0, span, 200)
    per_simd_end = {}
    for sid, ee in zip(simd[live], e[live]):
        per_simd_end[sid] = max(per_simd_end.get(sid, 0.0), ee)
    ends = np.array(sorted(per_simd_end.values()))
    conc = np.array([((s[live] <= g) & (e[live] > g)).sum() for g in grid]) / max(nsimd, 1)
    print("== %s: %d waves (%d with work) on %d SIMDs, span %.3f ms" % (tag, len(t), live.sum(), nsimd, span))
    print("   waves/SIMD: min %d mean %.2f max %d" % (cnt.min(), cnt.mean(), cnt.max()))
    print("   SIMD finish times (ms): p10 %.3f p50 %.3f p90 %.3f max %.3f"
          % tuple(np.percentile(ends, [10, 50, 90, 100])))
    print("   resident waves per SIMD over time (10 pts): %s"
          % " ".join("%.2f" % conc[i] for i in range(0, 200, 20)))
    print("   mean resident waves per SIMD over the span: %.2f" % conc.mean())
    it = iters[live]
    print("   wave work (sum lane iters): mean %.0f cv %.3f min %.0f max %.0f; max-lane/mean-lane %.3f"
          % (it.mean(), it.std() / it.mean(), it.min(), it.max(), (mx[live] * 64 / it).mean()))
    print("   wave duration ms: mean %.3f min %.3f max %.3f" % ((e - s)[live].mean(), (e - s)[live].min(),
                                                             (e - s)[live].max()))
    dur = (e - s)
    idx = np.argsort(-dur)[:8]
    wid = np.nonzero(t[:, 1] != 0)[0] if False else None
    print("   longest waves (start ms, duration ms, sum lane iters): %s" % ", ".join(
        "(%.2f, %.2f, %d)" % (s[i], dur[i], iters[i]) for i in idx))
    late = s > 0.5 * span
    print("   waves starting after half the span: %d, their mean duration %.3f ms (all: %.3f)"
          % (late.sum(), dur[late].mean() if late.any() else 0.0, dur.mean()))
    if save:
        os.makedirs(save, exist_ok=True)
        np.save(os.path.join(save, tag + ".npy"), t)


def main():
    save = None
    if "--save" in sys.argv:
        save = sys.argv[sys.argv.index("--save") + 1]
    dev = torch.device("cuda", 0)
    L = rtamd.lib()
    L.spt_trace_set.argtypes = [C.c_void_p]
    if os.environ.get("SCENE") == "c4":            # BASELINE configs[4] (hierarchy kernel)
        S, n, cam = rtamd.scenes.complex10k()
        rtamd.scenes.update_camera(cam, W, H)
    else:
        S, n = rtamd.scenes.cornell()
        cam = rtamd.scenes.cornell_camera(W, H)
    sc = rtamd.SmallptScene(S, n)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
    px = torch.zeros(W * H, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    run(L, sc, cam, seeds0, seeds, col, px, 0, H, st)          # warm-up
    for N in [int(v) for v in os.environ.get("NS", "1,2,4,8").split(",")]:
        r0, r1 = rdist.row_band(0 if N == 1 else N // 2, N, H)
        t, gx, gy = run(L, sc, cam, seeds0, seeds, col, px, r0, r1, st)
        analyse("N%d" % N, t, gx, gy, save)


if __name__ == "__main__":
    main()
