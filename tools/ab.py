"""A/B kernel timing of librt_hip.so builds under build_ab/<name>/ (one child
process per variant, interleaved rounds, HIP-event time on the launch stream).

    KERNEL=smallpt|whitted LIBS=a,b ROUNDS=2 REPS=5 python tools/ab.py

smallpt: Cornell 1920x1080, SPP (default 64) samples per launch (COUNT=full|rays: with counters); BAND=k/N renders
only row band k of N (rtamd.dist.row_band: the per-GPU work of an N-GPU frame).
whitted: raytracer3.0.06 scene, 1920x1080 (WH=640x480: configs[0]'s size), rows [20, H-70).
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))


def child():
    import numpy as np
    import torch
    import rtamd
    W, H = (int(v) for v in os.environ.get("WH", "1920x1080").split("x"))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    L = rtamd.lib()
    if os.environ.get("KERNEL", "smallpt") == "whitted":
        prims, n = rtamd.scenes.whitted_scene()
        nbytes = C.sizeof(prims)
        d_prims = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        d_prims.copy_(torch.frombuffer(bytearray(prims), dtype=torch.uint8))
        px = torch.zeros(W * H, dtype=torch.int32, device=dev)

        def run(warm=False):
            rtamd.check(L.rtw_render_async(d_prims.data_ptr(), n, px.data_ptr(), W, H, 20, H - 70, None,
                                           st.cuda_stream))
    else:
        SPP = int(os.environ.get("SPP", "64"))
        r0, r1 = 0, H
        if os.environ.get("BAND"):
            from rtamd import dist as rdist
            k, N = (int(v) for v in os.environ["BAND"].split("/"))
            r0, r1 = rdist.row_band(k, N, H)
        if os.environ.get("SCENE") == "c4":        # BASELINE configs[4] (8-wide hierarchy kernel)
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
        grp = os.environ.get("GROUP")              # k/N: the interleaved share of rank k of N
        # COUNT=full: all four counters (the counted kernel); COUNT=rays: calls and samples only
        cmode = os.environ.get("COUNT", "")
        cnt = torch.zeros(4, dtype=torch.int64, device=dev)
        cm = {"cptr": cnt.data_ptr() if cmode else None,
              "mode": rtamd.SPT_PATH_TRACING | (rtamd.SPT_COUNT_RAYS if cmode == "rays" else 0)}
        plain = os.environ.get("WARM_PLAIN")       # warm-up launches uncounted (they learn the tile order)

        def run(warm=False):
            mode, cptr = (0, None) if (warm and plain) else (cm["mode"], cm["cptr"])
            if grp:
                k, N = (int(v) for v in grp.split("/"))
                rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(),
                                                            seeds0.data_ptr(), seeds.data_ptr(), px.data_ptr(),
                                                            W, H, k, N, 0, SPP, mode, cptr, st.cuda_stream))
                return
            rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                 seeds.data_ptr(), px.data_ptr(), W, H, r0, r1, 0, SPP, mode,
                                                 cptr, st.cuda_stream))
    for _ in range(int(os.environ.get("WARM", "3" if os.environ.get("SCENE") == "c4" else "1"))):
        run(warm=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        run()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    if os.environ.get("PROF"):      # block counters of a tools-only instrumented build
        names = ["iter", "shadow", "nearest", "diff", "spec", "refr", "light", "bounce", "done",
                 "wcall", "wstep", "wleaf", "wshade"]
        buf = (C.c_ulonglong * (2 * len(names)))()
        L.spt_prof_read(buf)
        for b, nm in enumerate(names):
            lanes, waves = buf[2 * b], buf[2 * b + 1]
            print("  %-8s lanes %14d waves %12d lanes/wave-exec %.1f" % (nm, lanes, waves, lanes / max(waves, 1)))
    print("%s %s %s min %.3f med %.3f ms" % (os.environ.get("KERNEL", "smallpt"), os.environ.get("BAND", os.environ.get("GROUP", "")),
                                            os.environ.get("VARIANT", "?"), min(ts), float(np.median(ts))),
          flush=True)


def main():
    base = os.path.join(ROOT, "build_ab")
    libs = sorted(os.listdir(base)) if os.path.isdir(base) else []
    if os.environ.get("LIBS"):
        libs = os.environ["LIBS"].split(",")
    tree = os.path.join(ROOT, "se-195-project-ray-tracer_amd", "librt_hip.so")   # "main": the in-tree build
    variants = {name: {"RT_HIP_LIB": tree if name == "main" else os.path.join(base, name, "librt_hip.so")}
                for name in libs}
    if not variants:
        variants = {"tree": {}}
    for _ in range(int(os.environ.get("ROUNDS", "2"))):
        for name, env in variants.items():
            e = dict(os.environ, VARIANT=name, **env)
            subprocess.run([sys.executable, __file__, "child"], env=e, check=True, timeout=300)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        main()
