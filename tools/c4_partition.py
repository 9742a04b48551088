"""Single-GPU proxy of BASELINE configs[4] (10k-sphere scene, 1920x1080, 64
spp) split over N GPUs: per-rank render time, max over ranks, for

  * "interleaved": rank k renders the 8-row groups k, k+N, ...
    (spt_scene_render_groups_async, learnt heaviest-first order), and
  * "balanced": rank k renders its list of tile groups from
    rtamd.dist.balanced_partition over the per-group wave times of one
    learning frame (spt_scene_render_list_async) -- what bench.py's
    configs4_tiled line runs at N > 1.

Each rank's share runs alone on the one GPU (as it would on its own GPU),
after warm-up frames; median of REPS frames.  The N shares rendered into one
frame must equal the full-frame render bit for bit (checked).

    NS=4,8 REPS=5 python tools/c4_partition.py
    LIBS=a,b ROUNDS=2 QUICK=1 python tools/c4_partition.py   (A/B of build_ab/<lib> builds:
        one child process per lib and round; QUICK: balanced lists only)
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd import dist as rdist  # noqa: E402

W, H, SPP = 1920, 1080, int(os.environ.get("SPP", "64"))
REPS = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda", 0)
spheres, n, cam = rtamd.scenes.complex10k()
rtamd.scenes.update_camera(cam, W, H)
L = rtamd.lib()
st = torch.cuda.current_stream(dev)
seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
NG = rdist.group_count(W, H)


def bufs():
    return (torch.zeros(3 * W * H, dtype=torch.float32, device=dev), torch.empty_like(seeds0),
            torch.zeros(W * H, dtype=torch.int32, device=dev))


def timed(fn):
    ts = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), min(ts)


def render_list(sc, lst, col, sd, px, cost=None, flags=0):
    rtamd.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                              sd.data_ptr(), px.data_ptr(), W, H, lst.data_ptr(), lst.numel(), 0,
                                              SPP, flags, None, cost.data_ptr() if cost is not None else None,
                                              st.cuda_stream))


def render_groups(sc, k, N, col, sd, px):
    rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                sd.data_ptr(), px.data_ptr(), W, H, k, N, 0, SPP, 0, None,
                                                st.cuda_stream))


def main():
    if os.environ.get("LIBS") and not os.environ.get("C4_CHILD"):
        for r in range(int(os.environ.get("ROUNDS", "2"))):
            for lib in os.environ["LIBS"].split(","):
                path = os.path.join(ROOT, "build_ab", lib, "librt_hip.so") if lib != "main" else \
                    os.path.join(ROOT, "se-195-project-ray-tracer_amd", "librt_hip.so")
                print("--- lib %s round %d" % (lib, r), flush=True)
                subprocess.run([sys.executable, __file__], env=dict(os.environ, RT_HIP_LIB=path, C4_CHILD="1"),
                               check=True, timeout=600)
        return
    quick = os.environ.get("QUICK") == "1"
    sc_full = rtamd.SmallptScene(spheres, n)
    ref = bufs()
    for _ in range(3):
        rtamd.check(L.spt_scene_render_async(sc_full.handle, C.byref(cam), ref[0].data_ptr(), seeds0.data_ptr(),
                                             ref[1].data_ptr(), ref[2].data_ptr(), W, H, 0, H, 0, SPP, 0, None,
                                             st.cuda_stream))
    full_ms, _ = timed(lambda: rtamd.check(L.spt_scene_render_async(
        sc_full.handle, C.byref(cam), ref[0].data_ptr(), seeds0.data_ptr(), ref[1].data_ptr(), ref[2].data_ptr(),
        W, H, 0, H, 0, SPP, 0, None, st.cuda_stream)))
    print("full frame (1 GPU): %.2f ms" % full_ms, flush=True)
    for N in [int(v) for v in os.environ.get("NS", "4,8").split(",")]:
        # interleaved (one scene per rank: each learns its own order)
        res = []
        out = bufs()
        for k in (range(N) if not quick else []):
            sc = rtamd.SmallptScene(spheres, n)
            for _ in range(3):
                render_groups(sc, k, N, *out)
            res.append(timed(lambda: render_groups(sc, k, N, *out)))
            sc.close()
        if not quick:
            print("N=%d interleaved: per rank %s ms; max %.2f" % (N, [round(r[0], 2) for r in res],
                                                                   max(r[0] for r in res)), flush=True)
            ok = torch.equal(out[0].view(torch.int32), ref[0].view(torch.int32)) and torch.equal(out[2], ref[2])
            print("  assembled == full frame: %s" % ok, flush=True)
        # learning frame: interleaved lists with per-group costs
        cost = torch.zeros(NG, dtype=torch.int32, device=dev)
        sc = rtamd.SmallptScene(spheres, n)
        lists0 = [torch.tensor(rdist.interleaved_groups(k, N, W, H), dtype=torch.int32, device=dev) for k in range(N)]
        for k in range(N):
            render_list(sc, lists0[k], *bufs())                      # code objects, caches
        cost.zero_()
        for k in range(N):
            render_list(sc, lists0[k], *out, cost=cost)
        cmax = torch.zeros_like(cost)                            # each group's longest tile: the order key
        for k in range(N):
            render_list(sc, lists0[k], *bufs(), cost=cmax, flags=rtamd.SPT_COST_MAX)
        torch.cuda.synchronize()
        c = cost.cpu().numpy().astype(np.int64)
        parts = rdist.balanced_partition(c, N, order_key=None if os.environ.get("C4_SUM_ORDER") else
                                         cmax.cpu().numpy().astype(np.int64))
        print("  learnt costs: total %d ticks, max group %d, predicted per-rank loads %s" % (
            c.sum(), c.max(), [int(c[p].sum()) for p in parts]), flush=True)
        # SWEEP="n1:hw,..." times the balanced lists under other heavy-tile
        # policies (RT_SPT_TUNE coop = cooperative tiles, coop_waves = waves
        # per block that fetch them first); "-" = the library default.
        # TUNES="walk=32/16/32;coop=256" times them under whole RT_SPT_TUNE
        # strings instead (';'-separated).
        tune0 = os.environ.get("RT_SPT_TUNE")
        pols = os.environ["TUNES"].split(";") if os.environ.get("TUNES") else os.environ.get("SWEEP", "-").split(",")
        for pol in pols:
            if pol != "-" and "=" in pol:
                os.environ["RT_SPT_TUNE"] = pol + ("," + tune0 if tune0 else "")
            elif pol != "-":
                n1, hw = pol.split(":")
                os.environ["RT_SPT_TUNE"] = "coop=%s,coop_waves=%s" % (n1, hw) + ("," + tune0 if tune0 else "")
            else:
                os.environ.pop("RT_SPT_TUNE", None) if tune0 is None else os.environ.__setitem__("RT_SPT_TUNE", tune0)
            out = bufs()
            res = []
            for k in range(N):
                lst = torch.tensor(parts[k], dtype=torch.int32, device=dev)
                for _ in range(2):
                    render_list(sc, lst, *out)
                res.append(timed(lambda: render_list(sc, lst, *out)))
            print("N=%d balanced [%s]: per rank %s ms; max %.2f (min-of-reps max %.2f)" % (
                N, pol, [round(r[0], 2) for r in res], max(r[0] for r in res), max(r[1] for r in res)), flush=True)
            ok = torch.equal(out[0].view(torch.int32), ref[0].view(torch.int32)) and torch.equal(out[2], ref[2]) \
                and torch.equal(out[1], ref[1])
            print("  assembled == full frame: %s" % ok, flush=True)
        if tune0 is None:
            os.environ.pop("RT_SPT_TUNE", None)
        else:
            os.environ["RT_SPT_TUNE"] = tune0
        sc.close()


if __name__ == "__main__":
    main()
