"""The C++ drop-in shims driven by the reference apps' own launch sequences:
  * shim_whitted.cpp in place of openCLcode.cpp (testapp.cpp:57-178 order:
    openCLcode, AllocateBuffers, SetKernelArguments, Engine_InitRender,
    AllocateBuffers, SetKernelArguments, ExecuteKernel, ReadKernelBuffer);
  * shim_smallpt.cpp in place of smallptGPU.cpp (SetUpOpenCL -> SetUpHIP,
    then the idle loop's UpdateRenderingGPU calls).
Both must reproduce the CPU path exactly."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def _build():
    subprocess.run(["make", "-s", "-C", NATIVE, "apps"], check=True)


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


def test_smallpt_shim_matches_cpu_path(oracle, tmp_path):
    _build()
    w, h, passes = 320, 240, 5
    out = tmp_path / "state.bin"
    r = subprocess.run([os.path.join(NATIVE, "smallpt_app"), str(w), str(h), str(passes), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.uint32)
    px, col = raw[:w * h], raw[w * h:w * h * 4].view(np.float32)
    seeds0, cur = raw[w * h * 4:w * h * 6].copy(), int(raw[-1])
    assert cur == passes                      # < 20 passes: one sample per UpdateRenderingGPU
    assert (seeds0 >= 2).all()                # AllocateBuffers' clamp (smallptGPU.cpp:106-108)
    S, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    rc = np.zeros(3 * w * h, np.float32)
    seeds = seeds0.copy()
    rp = np.zeros(w * h, np.uint32)
    oracle.smallpt_render(S, n, cam, rc, seeds, rp, w, h, 0, cur, nthreads=8)
    assert (col.view(np.uint32) == rc.view(np.uint32)).all() and (px == rp).all()
