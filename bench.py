"""bench.py -- headline benchmark of the MI355X ray-trace hot path.

Workload (BASELINE.json metric "Mrays/sec + ms/frame @1920x1080 Cornell-64spp,
1/2/4/8 GPU; % HBM roofline"): one step = one 1920x1080 frame of the smallpt
Cornell scene (smallptgpu-v1.6/scene.h:29-40, reference camera) at 64
samples per pixel from the initial state (currentSample 0, AllocateBuffers'
glibc rand() seeds) -- RadiancePathTracing for every sample of every pixel,
running average, toInt pack -- plus, for N > 1, the RCCL all-gather that
assembles the HDR accumulator and the RGBA8 frame on every rank.

Rows are sharded over ranks in interleaved 8-row groups (rank k renders groups
k, k+N, ...: every GPU gets the same mix of the image; strong scaling: the
frame is fixed, each of N GPUs renders 1/N of it; RT_BENCH_BANDS=1: equal
contiguous bands instead); for N > 1 one RCCL all-gather of the HDR
accumulator per frame, then every rank repacks the RGBA8 frame from it
(spt_pack_pixels_async).  Frames are pipelined: frame
i+1 renders while frame i is gathered (double-buffered frame, second stream).
After the timed steps, rank 0's assembled frame is checked bit for bit
against one GPU rendering the whole frame ("frame_check").  Rays = Intersect +
IntersectP calls, counted by the kernel itself.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-whitted]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import glob
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (torch first: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

import rtamd  # noqa: E402
from rtamd import dist as rdist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: peak FP32 vector
W, H, SPP = 1920, 1080, 64


BENCH_KERNEL = "rt::smallpt::render_kernel<false, false, 0, true, false, 0>"   # the two-query (DUAL) kernel: Cornell has one light


def pmc_digest(kernel):
    """Per-launch PMC figures for `kernel` from the newest committed
    profiles/rNN/pmc_digest.json (written by tools/prof_round.sh +
    tools/pmc_digest.py from rocprofv3 --pmc passes of this bench command)."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_digest.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        # (kernel names with and without render_kernel's trailing CG = 0
        # argument, added in round 5, name the same kernel)
        norm = {k.replace(", 0>", ">"): k for k in d}
        key = kernel.replace(", 0>", ">")
        if key in norm:
            return d[norm[key]], os.path.relpath(f, ROOT)
    return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-whitted", action="store_true", help="skip the side lines")
    ap.add_argument("--no-cornell-extra", action="store_true",
                    help="skip the configs[2] / configs[3] lines (other launches of the headline kernel: "
                         "profiling runs keep its per-launch statistics to the headline frame)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU sample length")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle (C restatement, OpenMP over rows) on a bounded band of the same
    workload: rows of the 1920x1080 Cornell frame at 64 spp, sized to about
    args.cpu_seconds of host time."""
    import oracle_lib as O
    # OMP_NUM_THREADS is the host-CPU share of one GPU job on the MI355X pool
    # (16 of the node's 256 CPUs, set by the pool for every job); all 256 are
    # not ours to use.
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    S, n = O.cornell()
    cam = O.cornell_camera(W, H)
    col = np.zeros(3 * W * H, np.float32)
    px = np.zeros(W * H, np.uint32)
    seeds = O.seeds(W, H)
    # calibration band
    rows = max(threads, 8)
    r0 = H // 2 - rows // 2
    t0 = time.perf_counter()
    c = O.smallpt_render(S, n, cam, col, seeds.copy(), px, W, H, 0, SPP, row_begin=r0,
                         row_end=r0 + rows, nthreads=threads)
    dt = time.perf_counter() - t0
    rows2 = int(min(H, max(rows, rows * args.cpu_seconds / max(dt, 1e-3))))
    r0 = max(0, H // 2 - rows2 // 2)
    t0 = time.perf_counter()
    c = O.smallpt_render(S, n, cam, col, seeds.copy(), px, W, H, 0, SPP, row_begin=r0,
                         row_end=r0 + rows2, nthreads=threads)
    dt = time.perf_counter() - t0
    rays = c[0] + c[1]
    out = {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": "oracle/smallpt_oracle.c, rows [%d,%d) of the 1920x1080 Cornell frame at 64 spp "
                     "(%d samples, %.1f s, %d threads; %.3f Msamples/s)"
                     % (r0, r0 + rows2, c[3], dt, threads, c[3] / dt / 1e6),
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
           "cores_note": "OMP_NUM_THREADS: the pool's host-CPU share of a one-GPU job (16 of the node's CPUs)"}
    # The reference's own code (oracle/_ref: RadiancePathTracing & co. of
    # smallptgpu-v1.6 compiled from its sources) on one thread, as the
    # reference's CPU path runs; rays counted by the port on the same band
    # (identical work, checked bit for bit in tests/test_oracle.py).
    refs = O.ref_libs()
    if refs is not None:
        RS = refs[1]
        rows3, dt3 = 2, 0.0
        for _ in range(2):                  # probe, then a band sized to ~3 s
            if dt3:
                rows3 = int(min(H, max(rows3, rows3 * 3.0 / max(dt3, 1e-3))))
            r3 = H // 2 - rows3 // 2
            sd = seeds.copy()
            t0 = time.perf_counter()
            RS.ref_smallpt_render(S, n, C.byref(cam), col.ctypes.data, sd.ctypes.data, px.ctypes.data,
                                  W, H, r3, r3 + rows3, 0, SPP, 0)
            dt3 = time.perf_counter() - t0
        c3 = O.smallpt_render(S, n, cam, col, seeds.copy(), px, W, H, 0, SPP, row_begin=r3,
                              row_end=r3 + rows3, nthreads=threads)
        out["reference_1thread"] = {
            "value": round((c3[0] + c3[1]) / dt3 / 1e6, 3), "unit": "Mrays/s", "cores": 1, "kind": "reference",
            "sample": "oracle/_ref/libref_smallpt.so (the reference's geomfunc.h radiance), rows [%d,%d) of "
                      "the same frame at 64 spp, %.1f s, one thread" % (r3, r3 + rows3, dt3)}
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def whitted_line(args, dev):
    """Side line: BASELINE configs[1], Whitted 1920x1080 one frame on 1 GPU
    (device-resident frame, kernel timed with HIP events)."""
    prims, n = rtamd.scenes.whitted_scene()
    d_prims = torch.frombuffer(bytearray(bytes(prims)), dtype=torch.uint8).to(dev)
    frame = torch.zeros(W * H, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    L = rtamd.lib()

    def run(c):
        rtamd.check(L.rtw_render_async(d_prims.data_ptr(), n, frame.data_ptr(), W, H, 20, H - 70,
                                       c.data_ptr() if c is not None else None, s.cuda_stream))

    run(cnt)
    torch.cuda.synchronize(dev)
    counts = cnt.tolist()
    for _ in range(3):          # warm the uncounted kernels (first launches load their code objects)
        run(None)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record(s)
    for _ in range(reps):
        run(None)
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    rays = counts[0] + counts[1]
    out = {"workload": "Whitted raytracer3.0.06 scene 1920x1080, 9 primary rays/px, rows [20,1010)",
           "ms_per_frame": round(ms, 4), "Mrays_per_s": round(rays / ms / 1e3, 2),
           "rays_per_frame": rays, "ray_prim_tests": counts[2],
           "device_bytes": int(L.rt_cached_bytes())}
    if not args.no_cpu:
        import oracle_lib as O
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        _, c = O.whitted_render(W, H, row_begin=20, row_end=H - 70, nthreads=threads)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round((c[0] + c[1]) / dt / 1e6, 3), "unit": "Mrays/s",
                               "cores": threads, "kind": "port", "ms_per_frame": round(dt * 1e3, 1),
                               "sample": "oracle/whitted_oracle.c, the full frame"}
    return out


def configs0_line(args, dev):
    """Side line: BASELINE configs[0], the Whitted scene at 640x480 on the CPU
    path -- the reference's own timing loop (testapp.cpp:142-155: one
    Engine_InitRender + Engine_Render per run) restated by the oracle, on one
    thread as the reference runs and on the host share -- with the same frame
    on the GPU beside it."""
    import oracle_lib as O
    w, h = 640, 480
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    _, c = O.whitted_render(w, h, nthreads=1)
    dt1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.whitted_render(w, h, nthreads=threads)
    dtn = time.perf_counter() - t0
    rays = c[0] + c[1]
    prims, n = rtamd.scenes.whitted_scene()
    d_prims = torch.frombuffer(bytearray(bytes(prims)), dtype=torch.uint8).to(dev)
    frame = torch.zeros(w * h, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    L = rtamd.lib()
    run = lambda: rtamd.check(L.rtw_render_async(d_prims.data_ptr(), n, frame.data_ptr(), w, h, 20, h - 70,  # noqa: E731
                                                 None, s.cuda_stream))
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        run()
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / 10
    return {"workload": "configs[0]: Whitted raytracer3.0.06 scene 640x480, rows [20,410), CPU path",
            "rays_per_frame": rays,
            "cpu_1thread": {"ms_per_frame": round(dt1 * 1e3, 1), "Mrays_per_s": round(rays / dt1 / 1e6, 3),
                            "cores": 1, "kind": "port", "sample": "oracle/whitted_oracle.c, the full frame"},
            "cpu_threads": {"ms_per_frame": round(dtn * 1e3, 1), "Mrays_per_s": round(rays / dtn / 1e6, 3),
                            "cores": threads, "kind": "port", "sample": "oracle/whitted_oracle.c, the full frame"},
            "gpu": {"ms_per_frame": round(ms, 4), "Mrays_per_s": round(rays / ms / 1e3, 2)}}


def queue_line(args, dev):
    """Side line: the Raytracer3.2.03 queue tracer:
    raytracer_non_kernel's frame at the reference's own 800x600
    (raytracer.h:18-19) and at 1920x1080, one frame per launch sequence, HIP
    events; CPU baselines: the port on the host share and the reference's own
    raytracer_non_OpenCL.c (oracle/_ref) on one thread, both on the 800x600
    frame."""
    import oracle_lib as O
    prims, n = rtamd.scenes.queue_scene()
    d_prims = torch.frombuffer(bytearray(bytes(prims)[:96 * n]), dtype=torch.uint8).to(dev)
    L = rtamd.lib()
    s = torch.cuda.current_stream(dev)
    out = {"workload": "Raytracer3.2.03 queue tracer (raytracer_non_kernel), reference scene, 9 primary rays/px"}
    for w, h in [(800, 600), (W, H)]:
        frame = torch.zeros(w * h, dtype=torch.int32, device=dev)
        cnt = torch.zeros(4, dtype=torch.int64, device=dev)
        run = lambda c: rtamd.check(L.rtq_render_async(d_prims.data_ptr(), n, frame.data_ptr(), w, h, 0, h,  # noqa: E731
                                                       c.data_ptr() if c is not None else None, s.cuda_stream))
        run(cnt)
        torch.cuda.synchronize(dev)
        counts = cnt.tolist()
        for _ in range(3):      # warm the uncounted kernels (first launches load their code objects)
            run(None)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(s)
        for _ in range(reps):
            run(None)
        e1.record(s)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        rays = counts[0] + counts[1]
        out["%dx%d" % (w, h)] = {"ms_per_frame": round(ms, 4), "Mrays_per_s": round(rays / ms / 1e3, 2),
                                 "rays_per_frame": rays, "intersect_calls": counts[2],
                                 "device_bytes": int(L.rt_cached_bytes())}
    if not args.no_cpu:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        P, m = O.queue_scene()
        t0 = time.perf_counter()
        _, c = O.queue_render(800, 600, P, m, nthreads=threads)
        dt = time.perf_counter() - t0
        rays = c[0] + c[1]
        out["cpu_baseline"] = {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
                               "kind": "port", "ms_per_frame": round(dt * 1e3, 1),
                               "sample": "oracle/queue_oracle.c, the 800x600 frame"}
        Q = O.ref_queue_lib()
        if Q is not None:
            t0 = time.perf_counter()
            O.ref_queue_render(Q, 800, 600, P, m)
            dt = time.perf_counter() - t0
            out["reference_1thread"] = {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": 1,
                                        "kind": "reference", "ms_per_frame": round(dt * 1e3, 1),
                                        "sample": "oracle/_ref/libref_queue.so (the reference's own "
                                                  "raytracer_non_OpenCL.c), the 800x600 frame, one thread"}
    return out


def c5_line(args, dev):
    """Side line: BASELINE configs[4], the 10k-sphere scene_build_complex scene
    at 1920x1080, 64 spp, one frame on 1 GPU (the exact-culling hierarchy
    path), HIP events; CPU baseline on a band of rows at 1 spp."""
    spheres, n, cam = rtamd.scenes.complex10k()
    rtamd.scenes.update_camera(cam, W, H)
    sc = rtamd.SmallptScene(spheres, n)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
    px = torch.zeros(W * H, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    L = rtamd.lib()

    def run(c, mode=rtamd.SPT_PATH_TRACING):
        rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                             seeds.data_ptr(), px.data_ptr(), W, H, 0, H, 0, SPP,
                                             mode, c.data_ptr() if c is not None else None, s.cuda_stream))

    # Rays (Intersect + IntersectP calls) from a rays-only counted frame
    # (SPT_COUNT_RAYS: the uncounted walks); the reference's sphere-test count
    # from a full-counter frame (its shadow queries must find IntersectP's
    # early-exit position, the highest-index occluder).
    run(cnt, rtamd.SPT_PATH_TRACING | rtamd.SPT_COUNT_RAYS)
    torch.cuda.synchronize(dev)
    rays_counts = cnt.tolist()
    cnt.zero_()
    run(cnt)
    torch.cuda.synchronize(dev)
    counts = cnt.tolist()
    assert rays_counts[0] == counts[0] and rays_counts[1] == counts[1], (rays_counts, counts)
    # Steady state, as the headline steps: the first launches of a (window,
    # camera, spp) key record the tile groups' costs and build the
    # heaviest-first order (SptSched); then the median of three frames.
    for _ in range(2):
        run(None)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        run(None)
        e1.record(s)
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    rays = counts[0] + counts[1]
    out = {"workload": "configs[4]: scene_build_complex 10k spheres, 1920x1080, 64 spp, one frame "
                       "(median of 3 after 2 warm-up frames)",
           "ms_per_frame": round(ms, 3), "Mrays_per_s": round(rays / ms / 1e3, 2), "rays_per_frame": rays,
           "sphere_tests_reference": counts[2]}
    if not args.no_cpu:
        import oracle_lib as O
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        ccol = np.zeros(3 * W * H, np.float32)
        cpx = np.zeros(W * H, np.uint32)
        rows, dt = 8, 0.0
        for _ in range(2):                 # probe, then a band sized to ~3 s
            if dt:
                rows = int(min(H, max(rows, rows * 3.0 / max(dt, 1e-3))))
            r0 = H // 2 - rows // 2
            t0 = time.perf_counter()
            c = O.smallpt_render(spheres, n, cam, ccol, rtamd.scenes.seeds(W, H), cpx, W, H, 0, 1,
                                 row_begin=r0, row_end=r0 + rows, nthreads=threads)
            dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round((c[0] + c[1]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
                               "kind": "port", "sample": "oracle/smallpt_oracle.c (full scan), rows [%d,%d) at 1 spp, "
                               "%.1f s" % (r0, r0 + rows, dt)}
    return out


def cornell_line(args, dev, w, h, spp, workload):
    """Side lines: BASELINE configs[2] (Cornell 1024x768, 64 spp) and the
    per-GPU work of configs[3] (Cornell 1920x1080, 256 spp: one GPU renders
    the whole frame; the tiled 2/4/8-GPU form is the headline's sharded
    path) -- one launch per frame from the initial state, HIP events on the
    launch stream, median of 3 after a warm-up."""
    spheres, n = rtamd.scenes.cornell()
    cam = rtamd.scenes.cornell_camera(w, h)
    sc = rtamd.SmallptScene(spheres, n)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(w, h).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
    px = torch.zeros(w * h, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    L = rtamd.lib()

    def run(c=None):
        rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                             seeds.data_ptr(), px.data_ptr(), w, h, 0, h, 0, spp,
                                             rtamd.SPT_PATH_TRACING, c.data_ptr() if c is not None else None,
                                             s.cuda_stream))

    run(cnt)
    torch.cuda.synchronize(dev)
    counts = cnt.tolist()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        run()
        e1.record(s)
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    rays = counts[0] + counts[1]
    return {"workload": workload, "ms_per_frame": round(ms, 3), "Mrays_per_s": round(rays / ms / 1e3, 2),
            "Msamples_per_s": round(w * h * spp / ms / 1e3, 2), "rays_per_frame": rays}


def collective_name():
    """What carries the HDR all-gather at N > 1: RCCL (torch's "nccl" backend
    on ROCm) unless the one-GPU rehearsal knob RT_BENCH_BACKEND picked gloo."""
    return "RCCL" if os.environ.get("RT_BENCH_BACKEND", "nccl") == "nccl" else "gloo"


def dropin_line(args):
    """Side line: the reference's own host path over the drop-in --
    displayfunc.cpp's idle loop calling UpdateRenderingGPU (csrc/shim_smallpt.cpp
    in place of smallptGPU.cpp) on the Cornell frame at 1920x1080: 20 single
    passes, then time-boxed calls (smallptGPU.cpp:739-755) for ~3 s each way,
    samples/s as the reference's caption computes it (:777-781).  "batched":
    the shim's time box launches batches of passes (one wait per batch; the
    same per-pixel sample sequence); "per_pass": one launch and one wait per
    pass, as smallptGPU.cpp does (RT_SPT_SHIM_BATCH=1)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "native", "smallpt_dropin_bench")
    if not os.access(exe, os.X_OK):
        return {"skipped": "tests/native/smallpt_dropin_bench not built"}
    out = {"workload": "smallpt drop-in (shim_smallpt.cpp UpdateRenderingGPU), Cornell 1920x1080, "
                       "20 single passes then time-boxed calls"}
    for tag, env in (("batched", {}), ("per_pass", {"RT_SPT_SHIM_BATCH": "1"})):
        r = subprocess.run([exe, str(W), str(H), "3.0"], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, **env))
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        out[tag] = json.loads(line[-1]) if r.returncode == 0 and line else {"error": r.stderr[-300:]}
    return out


def tiled_line(step, cnt, dev, world, distributed, workload, spp, frames=2, warm=0, mode=0, **scene):
    """A frame of `workload` tiled across the job's GPUs exactly as the
    headline steps are (each rank renders its rows, then the RCCL all-gather
    + repack): a counted frame, `warm` untimed frames (hierarchy scenes learn
    their heaviest-first order over a key's first launches), then `frames`
    timed frames bracketed by barrier + synchronize, max over ranks."""
    cnt.zero_()
    step(counters=cnt, spp=spp, cmode=mode, **scene)
    for _ in range(warm):
        step(spp=spp, **scene)
    torch.cuda.synchronize(dev)
    counts = cnt.clone()
    if distributed:
        dist.all_reduce(counts)
    counts = counts.tolist()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(frames):
        step(spp=spp, **scene)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    ms = el * 1e3 / frames
    rays = counts[0] + counts[1]
    return {"workload": "%s, tiled across %d GPU(s)%s" % (
                workload, world, " + %s HDR all-gather" % collective_name() if world > 1 else ""),
            "n_gpus": world, "ms_per_frame": round(ms, 3), "Mrays_per_s": round(rays / ms / 1e3, 2),
            "Msamples_per_s": round(W * H * spp / ms / 1e3, 2), "rays_per_frame": rays}


def list_tiled_line(dev, rank, world, distributed, s, sc, cm, spp, workload, frames=3, warm=2):
    """BASELINE configs[4] at N > 1 split by measured cost: one learning frame
    renders the interleaved shares as tile-group lists recording every
    group's wave time (spt_scene_render_list_async), the costs are summed over
    the ranks (all-reduce), and every rank takes its list from the same
    deterministic longest-first partition (rtamd.dist.balanced_partition:
    each rank gets an equal share of the heaviest groups and of the total).
    Timed frames: render the list, then the group exchange (pack, one
    all-gather, unpack) and the RGBA8 repack on a second stream, overlapped
    with the next frame's render (double-buffered); barrier + synchronize
    around them, max over ranks."""
    L = rtamd.lib()
    ng = rdist.group_count(W, H)
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
    seeds = torch.empty_like(seeds0)
    cols = [torch.zeros(3 * W * H, dtype=torch.float32, device=dev) for _ in range(2)]
    pxs = [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(2)]
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    cost = torch.zeros(ng, dtype=torch.int32, device=dev)

    def render(lst, b, counters=None, cost_buf=None, flags=0):
        rtamd.check(L.spt_scene_render_list_async(
            sc.handle, C.byref(cm), cols[b].data_ptr(), seeds0.data_ptr(), seeds.data_ptr(), pxs[b].data_ptr(),
            W, H, lst.data_ptr(), lst.numel(), 0, spp, rtamd.SPT_PATH_TRACING | rtamd.SPT_COUNT_RAYS | flags,
            counters.data_ptr() if counters is not None else None,
            cost_buf.data_ptr() if cost_buf is not None else None, s.cuda_stream))

    mine0 = torch.tensor(rdist.interleaved_groups(rank, world, W, H), dtype=torch.int32, device=dev)
    render(mine0, 0, counters=cnt, cost_buf=cost)            # learning frame: costs + rays (rays-only mode)
    cost_max = torch.zeros_like(cost)                        # and each group's longest tile (the order key)
    render(mine0, 1, cost_buf=cost_max, flags=rtamd.SPT_COST_MAX)
    torch.cuda.synchronize(dev)
    costs = cost.to(torch.int64)
    keys = cost_max.to(torch.int64)
    counts = cnt.clone()
    if distributed:
        dist.all_reduce(costs)
        dist.all_reduce(keys)                                # (one rank renders each group: a sum is its value)
        dist.all_reduce(counts)
    costs = costs.cpu().numpy()
    keys = keys.cpu().numpy()
    counts = counts.tolist()
    parts = rdist.balanced_partition(costs, world, order_key=keys)
    mine = torch.tensor(parts[rank], dtype=torch.int32, device=dev)
    gs = torch.cuda.Stream(dev)

    def pack_groups(c, groups, n, buf):
        rtamd.check(L.spt_groups_pack_async(c.data_ptr(), W, H, groups.data_ptr(), n, buf.data_ptr(),
                                            torch.cuda.current_stream(dev).cuda_stream))

    def unpack_groups(c, groups, n, buf):
        rtamd.check(L.spt_groups_unpack_async(c.data_ptr(), W, H, groups.data_ptr(), n, buf.data_ptr(),
                                              torch.cuda.current_stream(dev).cuda_stream))

    def packer(b):
        return lambda: rtamd.check(L.spt_pack_pixels_async(cols[b].data_ptr(), pxs[b].data_ptr(), W, H, 0, H,
                                                           torch.cuda.current_stream(dev).cuda_stream))

    gathers = [rdist.ListGather(cols[b], pxs[b], rank, world, W, H, parts, pack=packer(b), pack_groups=pack_groups,
                                unpack_groups=unpack_groups) for b in range(2)]
    freed = [None, None]
    rev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(frames)]
    nf = [0]

    def frame(i=None):
        b = nf[0] % 2
        nf[0] += 1
        if freed[b] is not None:
            s.wait_event(freed[b])
        if i is not None:
            rev[i][0].record(s)
        render(mine, b, flags=rtamd.SPT_LIST_SET)          # (balanced_partition's lists are sets)
        if i is not None:
            rev[i][1].record(s)
        if world > 1:
            gs.wait_stream(s)
            with torch.cuda.stream(gs):
                gathers[b].gather()
            freed[b] = torch.cuda.Event()
            freed[b].record(gs)
        return b

    for _ in range(warm):
        frame()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = 0
    for i in range(frames):
        last = frame(i)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    render_ms = float(np.median([a.elapsed_time(b) for a, b in rev]))
    per_rank = [render_ms]
    if distributed:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        mine_t = torch.tensor([render_ms], dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine_t) for _ in range(world)]
        dist.all_gather(allr, mine_t)
        per_rank = [round(x.item(), 3) for x in allr]
    ms = el * 1e3 / frames
    rays = counts[0] + counts[1]
    out = {"workload": "%s, cost-balanced tile-group lists over %d GPU(s) + %s group all-gather" % (
               workload, world, collective_name()),
           "n_gpus": world, "ms_per_frame": round(ms, 3), "Mrays_per_s": round(rays / ms / 1e3, 2),
           "Msamples_per_s": round(W * H * spp / ms / 1e3, 2), "rays_per_frame": rays,
           "partition": "rtamd.dist.balanced_partition over one learning frame's per-group wave times (balanced "
                        "by their sum, each rank's list ordered by the group's longest tile: SPT_COST_MAX)",
           "render_ms_per_rank": per_rank,
           "predicted_load_per_rank": [int(costs[p].sum()) for p in parts]}
    # the assembled frame must equal one GPU rendering the whole frame
    ref_c = torch.zeros_like(cols[0])
    ref_p = torch.zeros_like(pxs[0])
    ref_s = torch.empty_like(seeds0)
    rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cm), ref_c.data_ptr(), seeds0.data_ptr(),
                                         ref_s.data_ptr(), ref_p.data_ptr(), W, H, 0, H, 0, spp,
                                         rtamd.SPT_PATH_TRACING, None, s.cuda_stream))
    torch.cuda.synchronize(dev)
    ok = torch.tensor([int(torch.equal(ref_c.view(torch.int32), cols[last].view(torch.int32))
                           and torch.equal(ref_p, pxs[last]))], dtype=torch.int32, device=dev)
    if distributed:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    out["frame_check"] = "assembled frame == single-GPU frame (bit-exact)" if ok.item() else "MISMATCH"
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    distributed = world > 1
    # Rehearsal knobs for a one-GPU box (never set by the driver):
    # RT_BENCH_BACKEND=gloo and RT_BENCH_SHARE_GPU=1 run N ranks on device 0.
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    gpu = local % torch.cuda.device_count() if os.environ.get("RT_BENCH_SHARE_GPU") else local
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        # Fail fast, with the collective library's own message, if the
        # communicator cannot be built or used: a short timeout and one tiny
        # all-reduce right after init (an RCCL failure otherwise surfaces
        # minutes later as a hang in the first frame's gather).
        import datetime
        try:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", gpu),
                                        timeout=datetime.timedelta(seconds=180))
            else:
                dist.init_process_group(backend, timeout=datetime.timedelta(seconds=180))
            probe = torch.ones(1, device=torch.device("cuda", gpu))
            dist.all_reduce(probe)
            torch.cuda.synchronize(gpu)
            if int(probe.item()) != world:
                raise RuntimeError("all-reduce probe returned %r, expected %d" % (probe.item(), world))
        except Exception as e:      # noqa: BLE001 -- reported verbatim, then exit non-zero
            print(json.dumps({"error": "collective init failed on rank %d (%s backend): %s: %s" % (
                rank, collective_name(), type(e).__name__, e)}), flush=True)
            sys.exit(3)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    rtamd.set_device(gpu)
    L = rtamd.lib()

    spheres, ns = rtamd.scenes.cornell()
    cam = rtamd.scenes.cornell_camera(W, H)
    scene = rtamd.SmallptScene(spheres, ns)       # uploaded once
    seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)  # pristine
    seeds = torch.empty_like(seeds0)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    interleaved = world > 1 and not os.environ.get("RT_BENCH_BANDS")
    r0, r1 = rdist.row_band(rank, world, H)
    B = len(rdist.group_rows(rank, world, H)) if interleaved else r1 - r0
    s = torch.cuda.current_stream(dev)
    # N > 1 over RCCL: frames are pipelined -- frame i+1 renders (stream s)
    # while frame i's HDR all-gather and RGBA8 repack run on a second stream,
    # with the frame buffers double-buffered (a buffer is rendered into again
    # only after its previous gather finished).  Each rank's progressive state
    # is its own band, so frame i+1 never needs frame i's gathered frame.
    pipelined = distributed and (backend == "nccl" or os.environ.get("RT_BENCH_PIPELINE") == "1") and \
        not os.environ.get("RT_BENCH_NO_PIPELINE")
    nbuf = 2 if pipelined else 1
    colors = [torch.zeros(3 * W * H, dtype=torch.float32, device=dev) for _ in range(nbuf)]
    pixels = [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(nbuf)]
    gs = torch.cuda.Stream(dev) if pipelined else s

    def packer(b):               # RGBA8 frame from the gathered HDR accumulator (toInt, bit-exact)
        def pack():
            rtamd.check(L.spt_pack_pixels_async(colors[b].data_ptr(), pixels[b].data_ptr(), W, H, 0, H,
                                                torch.cuda.current_stream(dev).cuda_stream))
        return pack

    Gather = rdist.GroupGather if interleaved else rdist.FrameGather
    gathers = [Gather(colors[b], pixels[b], rank, world, W, H, pack=packer(b)) for b in range(nbuf)]
    freed = [None] * nbuf        # event: buffer b's last gather finished
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]          # each timed step's all-gather + repack (gather stream)
    nframe = [0]

    def step(i=None, counters=None, spp=SPP, sc=None, cm=None, cmode=0):
        sc = scene if sc is None else sc
        cm = cam if cm is None else cm
        b = nframe[0] % nbuf
        nframe[0] += 1
        if freed[b] is not None:
            s.wait_event(freed[b])
        if i is not None:
            ev[i][0].record(s)
        cptr = counters.data_ptr() if counters is not None else None
        if interleaved:
            rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cm), colors[b].data_ptr(),
                                                        seeds0.data_ptr(), seeds.data_ptr(), pixels[b].data_ptr(),
                                                        W, H, rank, world, 0, spp, rtamd.SPT_PATH_TRACING | cmode,
                                                        cptr, s.cuda_stream))
        else:
            rtamd.check(L.spt_scene_render_async(sc.handle, C.byref(cm), colors[b].data_ptr(),
                                                 seeds0.data_ptr(), seeds.data_ptr(), pixels[b].data_ptr(), W, H,
                                                 r0, r1, 0, spp, rtamd.SPT_PATH_TRACING | cmode, cptr, s.cuda_stream))
        if i is not None:
            ev[i][1].record(s)
        if world > 1:            # RCCL all-gather of the HDR bands + RGBA8 repack
            gs.wait_stream(s)
            with torch.cuda.stream(gs):
                if i is not None:
                    gev[i][0].record(gs)
                gathers[b].gather()
                if i is not None:
                    gev[i][1].record(gs)
            if pipelined:
                freed[b] = torch.cuda.Event()
                freed[b].record(gs)

    for _ in range(args.warmup):
        step()
    cnt.zero_()
    step(counters=cnt)                      # one counted frame (counts are deterministic)
    torch.cuda.synchronize(dev)
    counts = cnt.clone()
    if distributed:
        dist.all_reduce(counts)
    counts = counts.tolist()
    rays_per_frame = counts[0] + counts[1]

    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ranks = None
    if distributed:
        # Per-rank view of the timed steps (HIP events): render kernel ms,
        # all-gather + repack ms on the gather stream, and this rank's wall
        # clock -- gathered so rank 0 can say which rank and which phase set
        # the frame time.
        gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gev]))
        mine = torch.tensor([kern_ms, gather_ms, elapsed * 1e3 / args.steps], dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        ranks = [r.tolist() for r in allr]
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = t.tolist()
    ms_per_step = elapsed * 1e3 / args.steps

    # The reference's frame ends in a blocking read of the pixels
    # (smallptGPU.cpp:760 ReadKernelBuffer after every pass): the same steps
    # again, each followed by a blocking D2H of the (assembled) RGBA8 frame
    # into page-locked host memory.  Reported beside ms_per_step (which keeps
    # the device-resident frame the driver's metric times).
    host_px = torch.empty(W * H, dtype=torch.int32, pin_memory=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        torch.cuda.synchronize(dev)                  # render (+ gather and repack on gs)
        host_px.copy_(pixels[(nframe[0] - 1) % nbuf], non_blocking=True)
        torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    rb = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([rb], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rb = t.item()
    ms_readback = rb * 1e3 / args.steps

    # Roofline: algorithmic HBM bytes of one launch =
    # 32 B per pixel of the band (seeds 8 in + 8 out, colour 12 out, pixel 4
    # out) + the scene (44 B per sphere).  The kernel is VALU-bound; the FP32
    # view counts 20 FLOP per ray-sphere test.
    launch_bytes = 32 * B * W + 44 * ns
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9
    flops = 20.0 * counts[2] / world
    pmc, pmc_src = pmc_digest(BENCH_KERNEL) if world == 1 else (None, None)
    out = {
        "metric": "Mrays/sec + ms/frame @1920x1080 Cornell-64spp, 1/2/4/8 GPU; % HBM roofline",
        "value": round(rays_per_frame / (ms_per_step * 1e-3) / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: reference Cornell scene (scene.h:29-40), glibc rand() seeds, random-free camera",
        "config": {"workload": "smallpt Cornell 1920x1080 64spp RadiancePathTracing, one frame per step",
                   "frame": [W, H], "spp": SPP, "spheres": ns, "rows_per_gpu": B,
                   "parallelism": ("%s x%d + %s HDR all-gather%s" % (
                       "interleaved 8-row groups" if interleaved else "row bands", world, collective_name(),
                       " (pipelined)" if pipelined else "")) if world > 1 else "single GPU"},
        "frames_per_s": round(1e3 / ms_per_step, 3),
        "ms_per_frame_with_readback": round(ms_readback, 3),
        "readback_note": "the same step followed by a blocking D2H of the %dx%d RGBA8 frame (%.1f MB) into "
                         "pinned host memory, as smallptGPU.cpp:760 reads after every pass; max over ranks" % (
                             W, H, W * H * 4 / 1e6),
        "Msamples_per_s": round(W * H * SPP / (ms_per_step * 1e-3) / 1e6, 2),
        "rays_per_frame": rays_per_frame,
        "kernel_ms": round(kern_ms, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": int(pmc["traffic_bytes"]) if pmc and "traffic_bytes" in pmc else None,
                     "traffic_source": pmc_src,
                     "algorithmic_bytes": launch_bytes,
                     "note": "compute-bound kernel: HBM roofline reported because the metric asks; "
                             "see valu"},
        "valu": {"achieved_tflops": round(flops / (kern_ms * 1e-3) / 1e12, 3),
                 "peak_tflops": FP32_PEAK_TFLOPS,
                 "frac": flops / (kern_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                 "basis": "20 FLOP per ray-sphere test",
                 "issue_frac": round(pmc["valu_issue_frac"], 4) if pmc and "valu_issue_frac" in pmc else None,
                 "lane_util": round(pmc["lane_util"], 4) if pmc and "lane_util" in pmc else None,
                 "issue_basis": "SQ_INSTS_VALU x 2 cycles (wave64 on SIMD32) / (1024 SIMDs x 2.4 GHz x "
                                "kernel time), from the PMC digest"},
    }
    if distributed:
        # Where the N-GPU frame time goes: with pipelining a step costs the
        # slowest rank's render when the gather hides behind the next frame's
        # render (overlap 1), render + gather when nothing overlaps (0).
        rmax = max(r[0] for r in ranks)
        gmax = max(r[1] for r in ranks)
        out["ranks"] = {"render_ms": [round(r[0], 3) for r in ranks],
                        "gather_ms": [round(r[1], 3) for r in ranks],
                        "wall_ms_per_step": [round(r[2], 3) for r in ranks],
                        "collective": collective_name(),
                        "overlap": round(min(1.0, max(0.0, (rmax + gmax - ms_per_step) / gmax)), 3) if gmax > 0 else None,
                        "note": "render_ms / gather_ms: mean over the timed steps of HIP events around the render "
                                "launch (render stream) and the HDR all-gather + RGBA8 repack (gather stream); "
                                "overlap = (max render + max gather - ms_per_step) / max gather"}
        # Self-check of the sharded path (outside the timed region): the last
        # assembled frame must equal one GPU rendering the whole frame.
        last = (nframe[0] - 1) % nbuf
        ref_c = torch.zeros_like(colors[0])
        ref_p = torch.zeros_like(pixels[0])
        ref_s = torch.empty_like(seeds0)
        rtamd.check(L.spt_scene_render_async(scene.handle, C.byref(cam), ref_c.data_ptr(), seeds0.data_ptr(),
                                             ref_s.data_ptr(), ref_p.data_ptr(), W, H, 0, H, 0, SPP,
                                             rtamd.SPT_PATH_TRACING, None, s.cuda_stream))
        torch.cuda.synchronize(dev)
        ok = torch.tensor([int(torch.equal(ref_c.view(torch.int32), colors[last].view(torch.int32))
                               and torch.equal(ref_p, pixels[last]))], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        out["frame_check"] = "assembled frame == single-GPU frame (bit-exact)" if ok.item() else "MISMATCH"
    if not args.no_whitted and not args.no_cornell_extra:
        out["configs3"] = tiled_line(step, cnt, dev, world, distributed, "configs[3]: Cornell 1920x1080, 256 spp", 256)
    if not args.no_whitted:
        c4s, c4n, c4cam = rtamd.scenes.complex10k()
        rtamd.scenes.update_camera(c4cam, W, H)
        c4scene = rtamd.SmallptScene(c4s, c4n)
        c4work = "configs[4]: 10k-sphere scene_build_complex, 1920x1080, 64 spp"
        if world > 1:
            out["configs4_tiled"] = list_tiled_line(dev, rank, world, distributed, s, c4scene, c4cam, SPP, c4work)
        else:
            out["configs4_tiled"] = tiled_line(step, cnt, dev, world, distributed, c4work, SPP, warm=2,
                                               sc=c4scene, cm=c4cam, mode=rtamd.SPT_COUNT_RAYS)
    if rank == 0 and world == 1:
        if not args.no_whitted:
            out["whitted"] = whitted_line(args, dev)
            out["configs4"] = c5_line(args, dev)
            out["queue3203"] = queue_line(args, dev)
            if not args.no_cornell_extra:
                out["configs2"] = cornell_line(args, dev, 1024, 768, 64, "configs[2]: Cornell 1024x768, 64 spp, 1 GPU")
                out["dropin"] = dropin_line(args)
            if not args.no_cpu:
                out["configs0"] = configs0_line(args, dev)
        out["cpu_baseline"] = None if args.no_cpu else cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
