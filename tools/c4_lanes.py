"""Where configs[4]'s lanes go (tools-only RT_SPT_TRACE build): per tile
(work item) the sum and the max over its 64 lanes of loop iterations.  A
wave runs its tile for max iterations while its lanes need sum / 64 on
average, so sum / (64 max) is the tile's lane efficiency from the tail of
uneven pixels alone (before any divergence inside an iteration).

    tools/build_variants.sh trace -DRT_SPT_TRACE
    RT_HIP_LIB=build_ab/trace/librt_hip.so python tools/c4_lanes.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import wave_trace as wt  # noqa: E402

rtamd = wt.rtamd


def main():
    import ctypes as C
    dev = torch.device("cuda", 0)
    L = rtamd.lib()
    L.spt_trace_set.argtypes = [C.c_void_p]
    S, n, cam = rtamd.scenes.complex10k()
    rtamd.scenes.update_camera(cam, wt.W, wt.H)
    sc = rtamd.SmallptScene(S, n)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(wt.W, wt.H).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * wt.W * wt.H, dtype=torch.float32, device=dev)
    px = torch.zeros(wt.W * wt.H, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    for rep in range(3):                                 # learn the order, then the measured frame
        t, gx, gy = wt.run(L, sc, cam, seeds0, seeds, col, px, 0, wt.H, st)
    t = t[t[:, 1] != 0]
    s, m = t[:, 4].astype(np.float64), t[:, 5].astype(np.float64)
    ok = m > 0
    s, m = s[ok], m[ok]
    print("tiles %d, iterations: lane sum %.4g, wave max-sum %.4g" % (len(s), s.sum(), m.sum()))
    print("tile-tail lane efficiency (sum / 64 max), time-weighted: %.3f" % (s.sum() / (64 * m.sum())))
    eff = s / (64 * m)
    for q in (10, 25, 50, 75, 90):
        print("  per-tile efficiency p%d: %.3f" % (q, np.percentile(eff, q)))
    order = np.argsort(-m)
    for frac in (0.01, 0.1, 0.5, 1.0):
        k = max(1, int(len(m) * frac))
        sel = order[:k]
        print("  heaviest %4.0f%% of tiles: %.1f%% of wave iterations, efficiency %.3f" % (
            100 * frac, 100 * m[sel].sum() / m.sum(), s[sel].sum() / (64 * m[sel].sum())))
    ph = t[ok]
    print("walk cycles / total cycles (max lane, per tile): %.3f" % (ph[:, 8].astype(float).sum() / ph[:, 7].astype(float).sum()))
    print("leaf cycles / walk cycles: %.3f" % (ph[:, 9].astype(float).sum() / ph[:, 8].astype(float).sum()))


if __name__ == "__main__":
    main()
