"""Phase stamps of the configs[4] hierarchy kernel's heaviest waves (tools-only
RT_SPT_TRACE build): per wave the cycles spent walking the hierarchy (and in
its leaf blocks) against the rest of the loop (shading), walk trips, leaf
passes, queries and loop iterations -- at the window of rank k of N
(interleaved 8-row groups, as bench.py shards the frame), then the heaviest
tile group rendered ALONE on the chip (spt_trace_only_group), which splits
co-resident contention from the chain's own latency.

    tools/build_variants.sh trace -DRT_SPT_TRACE
    RT_HIP_LIB=build_ab/trace/librt_hip.so N=8 K=0 python tools/c5_phase.py
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402

W, H, SPP = 1920, 1080, int(os.environ.get("SPP", "64"))
N = int(os.environ.get("N", "1"))
KS = [int(v) for v in os.environ.get("K", "0").split(",")]   # ranks to trace (K=0,1,...)


def main():
    dev = torch.device("cuda", 0)
    L = rtamd.lib()
    L.spt_trace_set.argtypes = [C.c_void_p]
    L.spt_trace_only_group.argtypes = [C.c_int]
    S, n, cam = rtamd.scenes.complex10k()
    rtamd.scenes.update_camera(cam, W, H)
    sc = rtamd.SmallptScene(S, n)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
    px = torch.zeros(W * H, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    nw = (((W + 7) // 8) * ((H + 7) // 8) + 64) * 8    # work items (upper bound: tiles split up to 8 ways)
    buf = torch.zeros(nw * 16, dtype=torch.int32, device=dev)

    K = [0]

    def launch():
        rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                    seeds.data_ptr(), px.data_ptr(), W, H, K[0], N, 0, SPP, 0, None,
                                                    st.cuda_stream))

    def traced(tag):
        buf.zero_()
        rtamd.check(L.spt_trace_set(C.c_void_p(buf.data_ptr())))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        launch()
        b.record(st)
        torch.cuda.synchronize()
        rtamd.check(L.spt_trace_set(None))
        t = buf.cpu().numpy().view(np.uint32).reshape(nw, 16).astype(np.int64)
        t = t[t[:, 1] != 0]
        t0, t1 = t[:, 0], np.where(t[:, 1] < t[:, 0], t[:, 1] + (1 << 32), t[:, 1])
        dur = (t1 - t0) * 1e-5                           # ms (100 MHz)
        it_sum, it_max, grp, tot = t[:, 4], t[:, 5], t[:, 6], t[:, 7]
        walk, leaf, trips, lruns, queries = t[:, 8], t[:, 9], t[:, 10], t[:, 11], t[:, 12]
        live = it_sum > 0
        print("== %s: kernel %.2f ms (HIP events), %d waves with work, span %.2f ms" % (
            tag, a.elapsed_time(b), live.sum(), (t1[live].max() - t0[live].min()) * 1e-5))
        ghz = tot[live] / np.maximum(dur[live], 1e-9) * 1e-6
        print("   s_memtime rate: %.2f GHz median (cycles / wall)" % np.median(ghz))
        idx = np.argsort(-dur * live)[:8]
        print("   heaviest waves: grp dur_ms iters(max lane) walk%% leaf%% shade%% cyc/iter walk_cyc/query trips/query "
              "leafpass/query queries")
        for i in idx:
            q = max(queries[i], 1)
            print("     %5d %6.2f %6d %5.1f %5.1f %5.1f %7.0f %7.0f %6.1f %5.1f %6d" % (
                grp[i], dur[i], it_max[i], 100.0 * walk[i] / tot[i], 100.0 * leaf[i] / tot[i],
                100.0 * (tot[i] - walk[i]) / tot[i], tot[i] / max(it_max[i], 1), walk[i] / q, trips[i] / q,
                lruns[i] / q, queries[i]))
        ww = live
        print("   all waves: walk %.1f%% (leaf %.1f%%) of wave cycles; per query %.1f trips, %.1f leaf passes; "
              "mean cyc/iter %.0f" % (100.0 * walk[ww].sum() / tot[ww].sum(), 100.0 * leaf[ww].sum() / tot[ww].sum(),
                                     trips[ww].sum() / queries[ww].sum(), lruns[ww].sum() / queries[ww].sum(),
                                     (tot[ww] / np.maximum(it_max[ww], 1)).mean()))
        return grp[idx[0]], dur[idx[0]]

    worst = None
    for k in KS:
        K[0] = k
        launch()
        launch()
        torch.cuda.synchronize()                         # adaptive order learnt
        g, d = traced("configs[4] window %d/%d, %d spp" % (k, N, SPP))
        if worst is None or d > worst[2]:
            worst = (k, g, d)
    K[0] = worst[0]
    launch()
    torch.cuda.synchronize()
    rtamd.check(L.spt_trace_only_group(int(worst[1])))
    try:
        traced("window %d/%d: its heaviest group %d alone" % (worst[0], N, worst[1]))
    finally:
        rtamd.check(L.spt_trace_only_group(-1))


if __name__ == "__main__":
    main()
