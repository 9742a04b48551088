"""The C++ drop-in shims driven by the reference apps' own launch sequences:
  * shim_whitted.cpp in place of openCLcode.cpp (testapp.cpp:57-178 order:
    openCLcode, AllocateBuffers, SetKernelArguments, Engine_InitRender,
    AllocateBuffers, SetKernelArguments, ExecuteKernel, ReadKernelBuffer);
  * shim_smallpt.cpp in place of smallptGPU.cpp (SetUpOpenCL -> SetUpHIP,
    then the idle loop's UpdateRenderingGPU calls);
  * shim_queue.cpp in place of Raytracer3.2.03's raytracer_non_OpenCL.c
    (raytracer.c's main() with the reference's own scene.c / bitmap.c).
All must reproduce the CPU path exactly."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def _build():
    subprocess.run(["make", "-s", "-C", NATIVE, "apps"], check=True)


def _ref_app(name):
    """A harness linking the reference's own sources: built where
    /root/reference exists and shipped prebuilt; absent on a fresh checkout
    without the reference, where its tests skip."""
    path = os.path.join(NATIVE, name)
    if not os.access(path, os.X_OK):
        pytest.skip("%s not built (needs /root/reference)" % name)
    return path


def test_whitted_shim_matches_cpu_path(oracle, tmp_path):
    _build()
    w, h = 800, 600
    out = tmp_path / "frame.bin"
    r = subprocess.run([os.path.join(NATIVE, "whitted_app"), str(w), str(h), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.uint32).reshape(h, w)
    ref, _ = oracle.whitted_render(w, h, nthreads=8)
    assert (got == ref).all()


def test_whitted_shim_opencl_semantics(oracle, tmp_path):
    """RT_WHITTED_SEMANTICS=opencl: the shim computes raytrace_kernel's frame."""
    _build()
    w, h = 800, 600
    out = tmp_path / "frame.bin"
    env = dict(os.environ, RT_WHITTED_SEMANTICS="opencl")
    r = subprocess.run([os.path.join(NATIVE, "whitted_app"), str(w), str(h), str(out)],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.uint32).reshape(h, w)
    ref, _ = oracle.whitted_render_ocl(w, h, nthreads=8)
    assert (got[20:530] == ref[20:530]).all()


@pytest.mark.parametrize("w,h", [(800, 600), (640, 480)])
def test_whitted_shim_with_reference_scene_and_surface(oracle, tmp_path, w, h):
    """testapp.cpp:57-136's OpenCL sequence with the reference's own scene.cpp
    (Engine_Constructor's Scene, TracedRays_init, Scene_InitScene and the
    m_* globals) and surface.cpp (Surface_Create / Surface_Clear) linked in
    (800x600 = SCRWIDTH x SCRHEIGHT, testapp.cpp:18-19): the window rows are
    the CPU path's image, every other row keeps the cleared value."""
    _build()
    out = tmp_path / "frame.bin"
    r = subprocess.run([_ref_app("whitted_ref_app"), str(w), str(h), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.uint32).reshape(h, w)
    ref, _ = oracle.whitted_render(w, h, nthreads=8)
    assert (got[20:h - 70] == ref[20:h - 70]).all()
    assert not got[:20].any() and not got[h - 70:].any()


# RT_SPT_DEVICES: the drop-in tiles the frame over these devices; "0,0,0"
# runs the multi-GPU band / assemble code with three bands on one GPU.
BANDS = [pytest.param({}, id="one_band"), pytest.param({"RT_SPT_DEVICES": "0,0,0"}, id="three_bands")]


def _smallpt_app(tmp_path, w, h, passes, env, script=None):
    _build()
    out = tmp_path / "state.bin"
    cmd = [os.path.join(NATIVE, "smallpt_app"), str(w), str(h), str(passes), str(out)]
    if script:
        cmd.append(script)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.uint32)
    n = w * h
    st = {"pixels": raw[:n], "colors": raw[n:4 * n].view(np.float32), "seeds0": raw[4 * n:6 * n].copy(),
          "current": int(raw[6 * n]), "bands": int(raw[6 * n + 1]), "after": [int(v) for v in raw[6 * n + 2:]]}
    return st


@pytest.mark.parametrize("env", BANDS)
def test_smallpt_shim_matches_cpu_path(oracle, tmp_path, env):
    w, h, passes = 320, 240, 5
    st = _smallpt_app(tmp_path, w, h, passes, env)
    assert st["bands"] == (3 if env else 1)
    assert st["current"] == passes            # < 20 passes: one sample per UpdateRenderingGPU
    assert (st["seeds0"] >= 2).all()          # AllocateBuffers' clamp (smallptGPU.cpp:106-108)
    S, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    rc = np.zeros(3 * w * h, np.float32)
    seeds = st["seeds0"].copy()
    rp = np.zeros(w * h, np.uint32)
    oracle.smallpt_render(S, n, cam, rc, seeds, rp, w, h, 0, st["current"], nthreads=8)
    assert (st["colors"].view(np.uint32) == rc.view(np.uint32)).all() and (st["pixels"] == rp).all()


@pytest.mark.parametrize("env", BANDS)
def test_smallpt_shim_batched_passes(oracle, tmp_path, env):
    """Past 20 samples UpdateRenderingGPU runs time-boxed batches
    (smallptGPU.cpp:739-755): 20 single passes, then calls that each run as
    many passes as fit 0.5 * min(currentSample - 20, 100) / 100 s."""
    w, h = 160, 120
    st = _smallpt_app(tmp_path, w, h, 0, env, "p20,p1,p1,p1")
    a = st["after"]
    assert a[0] == 20 and a[1] == 21          # threshold 0 s: exactly one pass
    assert a[3] > a[2] > a[1]                 # batches grow with the sample count
    S, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    rc = np.zeros(3 * w * h, np.float32)
    seeds = st["seeds0"].copy()
    rp = np.zeros(w * h, np.uint32)
    oracle.smallpt_render(S, n, cam, rc, seeds, rp, w, h, 0, st["current"], nthreads=8)
    assert (st["colors"].view(np.uint32) == rc.view(np.uint32)).all() and (st["pixels"] == rp).all()


@pytest.mark.parametrize("env", BANDS)
def test_smallpt_shim_reinit(oracle, tmp_path, env):
    """ReInitGPU(1) (FreeBuffers + AllocateBuffers: new rand() seeds, the
    sample count restarts), ReInitGPU(0) (restart, RNG words continue) and
    ReInitSceneGPU after an edited sphere (smallptGPU.cpp:784-830)."""
    w, h = 160, 120
    S, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    # ReInitGPU(1) after 3 passes: the final state is 2 passes from the new seeds.
    st = _smallpt_app(tmp_path, w, h, 0, env, "p3,R,p2")
    assert st["after"] == [3, 0, 2]
    rc, rp, seeds = np.zeros(3 * w * h, np.float32), np.zeros(w * h, np.uint32), st["seeds0"].copy()
    oracle.smallpt_render(S, n, cam, rc, seeds, rp, w, h, 0, 2, nthreads=8)
    assert (st["colors"].view(np.uint32) == rc.view(np.uint32)).all() and (st["pixels"] == rp).all()
    # ReInitGPU(0) and ReInitSceneGPU: the RNG chain continues across the restart.
    for script, edit in (("p3,r,p2", False), ("p4,S,p3", True)):
        st = _smallpt_app(tmp_path, w, h, 0, env, script)
        k1, k2 = int(script[1]), int(script[-1])
        assert st["after"] == [k1, 0, k2]
        S2, n2 = oracle.cornell()
        rc, rp, seeds = np.zeros(3 * w * h, np.float32), np.zeros(w * h, np.uint32), st["seeds0"].copy()
        oracle.smallpt_render(S2, n2, cam, rc, seeds, rp, w, h, 0, k1, nthreads=8)
        if edit:
            S2[6].p.x += np.float32(1.0)
        oracle.smallpt_render(S2, n2, cam, rc, seeds, rp, w, h, 0, k2, nthreads=8)
        assert (st["colors"].view(np.uint32) == rc.view(np.uint32)).all() and (st["pixels"] == rp).all(), script


def test_smallpt_drop_in_main(oracle, tmp_path):
    """The drop-in's own main / mainGPU (shim_smallpt_main.cpp,
    smallptGPU.cpp:832-884) at displayfunc.cpp's default 640x480, with a GLUT
    stand-in whose main loop runs the idle callback three times."""
    _build()
    out = tmp_path / "main.bin"
    env = dict(os.environ, RT_TEST_PASSES="3", RT_TEST_OUT=str(out))
    r = subprocess.run([os.path.join(NATIVE, "smallpt_main_app")], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stderr
    w, h = 640, 480
    raw = np.fromfile(out, dtype=np.uint32)
    px, cur, seeds0 = raw[:w * h], int(raw[w * h]), raw[w * h + 1:].copy()
    assert cur == 3 and seeds0.size == 2 * w * h
    S, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    rc, rp = np.zeros(3 * w * h, np.float32), np.zeros(w * h, np.uint32)
    oracle.smallpt_render(S, n, cam, rc, seeds0, rp, w, h, 0, 3, nthreads=8)
    assert (px == rp).all()


@pytest.mark.parametrize("w,h", [(800, 600), (640, 480)])
def test_queue_shim_writes_the_reference_bmp(oracle, tmp_path, w, h):
    """Raytracer3.2.03's main() sequence (create_scene, Primitive_2 copy,
    raytracer_non_kernel -> the GPU, write_bmp_file) with the reference's own
    scene.c and bitmap.c: at 800 x 600 (raytracer.h:18-19) the file is the
    reference's committed test.bmp, byte for byte."""
    import hashlib
    import json
    import rtamd.bmp
    _build()
    out = tmp_path / "test.bmp"
    r = subprocess.run([_ref_app("queue_ref_app"), str(w), str(h), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    data = out.read_bytes()
    if (w, h) == (800, 600):
        ka = json.load(open(os.path.join(os.path.dirname(NATIVE), "golden", "known_answers.json")))
        assert hashlib.sha256(data).hexdigest() == ka["queue3203"]["test_bmp"]["sha256"]
    ref, _ = oracle.queue_render(w, h, nthreads=8)
    assert data == rtamd.bmp.bmp_bytes(ref)
