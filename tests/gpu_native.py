"""ctypes driver for tests/native/libgpu_math_check.so (test infrastructure)."""
import ctypes as C
import os
import subprocess

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")

# (name, fn id, lo, hi) float-bit ranges: the hot path's input domains.
DOMAINS = [
    ("powf_y20", 0, 0x00000000, 0x40000000),     # raytracer.cpp:165, dot in (0, 2]
    ("powf_gamma", 1, 0x00000000, 0x3f800000),   # vec.h:62, [0, 1]
    ("powf_gamma_negzero", 1, 0x80000000, 0x80000000),
    ("expf_all", 2, 0x00000000, 0xffffffff),     # raytracer.cpp:487-489
    ("sinf", 3, 0x00000000, 0x41000000),         # geomfunc.h:66,262, [0, 8]
    ("cosf", 4, 0x00000000, 0x41000000),         # geomfunc.h:65,261
    ("sincosf_sin", 5, 0x00000000, 0x41000000),  # branch-free pair used by smallpt.hip
    ("sincosf_cos", 6, 0x00000000, 0x41000000),
    ("sincosf_sin_neg", 5, 0x80000000, 0xc1000000),
    ("sincosf_cos_neg", 6, 0x80000000, 0xc1000000),
    ("sqrt_rn_pos", 7, 0x00000000, 0x7fffffff),  # rt_common.h sqrt_rn: every non-negative float, NaNs
    ("sqrt_rn_neg", 7, 0x80000000, 0xffffffff),  # every negative float (NaN results, -0)
    # rt_common.h short forms: sqrt_nr / rcp_nr on their stated ranges, and the
    # guarded sqrt_exact / inv_len (uniform fallback) on every float
    ("sqrt_nr_range", 11, 0x0f800000, 0x7f7fffff),   # [2^-96, FLT_MAX]
    ("rcp_nr_range", 10, 0x00800000, 0x7c7fffff),    # [2^-126, 2^126)
    ("rcp_nr_range_neg", 10, 0x80800000, 0xfc7fffff),
    ("sqrt_exact_all", 8, 0x00000000, 0xffffffff),
    ("inv_len_all", 9, 0x00000000, 0xffffffff),
]


def lib():
    path = os.path.join(HERE, "libgpu_math_check.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", HERE, "libgpu_math_check.so"], check=True)
    L = C.CDLL(path)
    L.gmc_run.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    L.gmc_run_pow20.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    return L


def pow20_check(lo=0x00000001, hi=0x40800000):
    """rtm::pow_d(x, 20.0) on the device vs the host glibc pow for every float
    x with bits in [lo, hi] (default: (0, 4]); (count, mismatches, first bad)."""
    L = lib()
    bad, first = C.c_uint64(), C.c_uint32()
    rc = L.gmc_run_pow20(lo, hi, C.byref(bad), C.byref(first))
    if rc != 0:
        raise RuntimeError("gmc_run_pow20 failed (%d)" % rc)
    return hi - lo + 1, bad.value, hex(first.value)


def math_check(domains=DOMAINS):
    L = lib()
    out = {}
    for name, fn, lo, hi in domains:
        bad, first = C.c_uint64(), C.c_uint32()
        rc = L.gmc_run(fn, lo, hi, C.byref(bad), C.byref(first))
        if rc != 0:
            raise RuntimeError("gmc_run failed (%d) on %s" % (rc, name))
        out[name] = (hi - lo + 1, bad.value, hex(first.value))
    return out
