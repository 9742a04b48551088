"""GPU check of rt_glibc_math.h: device powf/expf/sinf/cosf (v_fma_f64 ...)
vs the host glibc, exhaustively over the hot path's input domains."""
import pytest

pytestmark = pytest.mark.gpu


def test_device_math_matches_host_glibc():
    import gpu_native
    res = gpu_native.math_check()
    bad = {k: v for k, v in res.items() if v[1] != 0}
    assert not bad, bad


def test_device_pow_d_matches_host_glibc():
    """The 3.2.03 queue tracer's pow(float, 20) (g++: glibc double pow)."""
    import gpu_native
    n, bad, first = gpu_native.pow20_check()
    assert n > 1.08e9 and bad == 0, (bad, first)
