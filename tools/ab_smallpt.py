"""A/B timing of smallpt kernel variants in one process per variant set
(interleaved rounds; HIP-event kernel time of the 1920x1080 64 spp frame)."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    import numpy as np
    import torch
    import rtamd
    W, H, SPP = 1920, 1080, int(os.environ.get("SPP", "64"))
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

    def run():
        rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                             seeds.data_ptr(), px.data_ptr(), W, H, 0, H, 0, SPP, 0, None,
                                             st.cuda_stream))
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st); run(); b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print("%s %.3f %.3f" % (os.environ.get("VARIANT", "?"), min(ts), float(np.median(ts))), flush=True)
    sys.exit(0)

variants = {}
libs = sorted(os.listdir(os.path.join(ROOT, "build_ab"))) if os.path.isdir(os.path.join(ROOT, "build_ab")) else []
for lib_name in (os.environ.get("LIBS", ",".join(libs)).split(",") if libs else []):
    path = os.path.join(ROOT, "build_ab", lib_name, "librt_hip.so")
    variants[lib_name + "/fixed9"] = {"RT_HIP_LIB": path}
    variants[lib_name + "/dyn"] = {"RT_HIP_LIB": path, "RT_SPT_NOFIX": "1"}
if not variants:
    variants = {"fixed9": {}, "dyn_lds": {"RT_SPT_NOFIX": "1"}}
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for name, env in variants.items():
        e = dict(os.environ, VARIANT=name, **env)
        subprocess.run([sys.executable, __file__, "child"], env=e, check=True)
