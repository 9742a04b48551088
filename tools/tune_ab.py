"""A/B of launch tunings (RT_SPT_TUNE strings) on BASELINE configs[4]
(10k-sphere scene, 1920x1080, 64 spp from the initial state) in one process:
per tuning, warm frames (the first records the tile costs, the learnt order
applies from the next), then REPS timed frames (HIP events, median and min),
each frame checked against the reference-core golden hashes.  GROUP=k/N
times an interleaved share instead of the full frame; COUNTED=1 times the
full-counter kernels (all four reference counters).

    TUNES="-;coop=512;walk=8/16/32" REPS=5 python tools/tune_ab.py   ("-": the defaults)
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "se-195-project-ray-tracer_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402
import oracle_lib  # noqa: E402

W, H, SPP = int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080)), int(os.environ.get("SPP", 64))
REPS, WARM = int(os.environ.get("REPS", 5)), int(os.environ.get("WARM", 3))
TUNES = os.environ.get("TUNES", "-").split(";")
GROUP = os.environ.get("GROUP")
COUNTED = os.environ.get("COUNTED") == "1"
dev = torch.device("cuda", 0)
spheres, n, cam = rtamd.scenes.complex10k()
rtamd.scenes.update_camera(cam, W, H)
gold = None
if (W, H, SPP) == (1920, 1080, 64) and not GROUP:
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "known_answers.json")))["smallpt"][
        "1920x1080_64spp_complex10k"]
seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
L = rtamd.lib()
st = torch.cuda.current_stream(dev)
ref = None
for tune in TUNES:
    os.environ["RT_SPT_TUNE"] = "" if tune == "-" else tune
    sc = rtamd.SmallptScene(spheres, n)              # (a fresh scene: its own learnt order)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
    px = torch.zeros(W * H, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    cptr = C.cast(C.c_void_p(cnt.data_ptr()), C.POINTER(C.c_uint64)) if COUNTED else None

    def run():
        if GROUP:
            k, N = (int(v) for v in GROUP.split("/"))
            rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                        seeds.data_ptr(), px.data_ptr(), W, H, k, N, 0, SPP, 0, cptr,
                                                        st.cuda_stream))
        else:
            rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                 seeds.data_ptr(), px.data_ptr(), W, H, 0, H, 0, SPP, 0, cptr,
                                                 st.cuda_stream))

    for _ in range(WARM):
        run()
    torch.cuda.synchronize()
    ts = []
    ok = True
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
        c, p, s = col.cpu().numpy(), px.cpu().numpy().view(np.uint32), seeds.cpu().numpy().view(np.uint32)
        h = (oracle_lib.fnv1a64(c), oracle_lib.fnv1a64(p), oracle_lib.fnv1a64(s))
        if gold is not None:
            ok = ok and h == (gold["colors"], gold["pixels"], gold["seeds"])
        else:
            ref = ref or h
            ok = ok and h == ref
    print("tune=%-40s median %.3f ms  min %.3f ms  %s  [%s]" % (
        tune, float(np.median(ts)), min(ts), "EXACT" if ok else "MISMATCH", " ".join("%.2f" % t for t in ts)),
        flush=True)
    sc.close()
