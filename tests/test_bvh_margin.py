"""Empirical check of the error bound behind the sphere hierarchy's culling
margin (smallpt.hip, BvhView comment): for grazing rays the point at the
float32 SphereIntersect distance (geomfunc.h:32-59 arithmetic, no FMA) lies
within 1.04e-3 * max(|op|, r) of the sphere (the analytical bound), far below
the 1/128 the traversal uses."""
import numpy as np


def test_float_root_within_margin_bound():
    rng = np.random.default_rng(7)
    n = 400_000
    f = np.float32
    c = rng.uniform(-300, 300, (n, 3)).astype(f)
    r = (10 ** rng.uniform(-2, 3, n)).astype(f)
    o = rng.uniform(-300, 300, (n, 3)).astype(f)
    u = rng.standard_normal((n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    tgt = c.astype(np.float64) + r[:, None] * (1 + rng.uniform(-1e-3, 1e-3, n))[:, None] * u
    d = tgt - o.astype(np.float64)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(f)
    op = (c - o).astype(f)
    b = ((op[:, 0] * d[:, 0] + op[:, 1] * d[:, 1]).astype(f) + op[:, 2] * d[:, 2]).astype(f)
    oo = ((op[:, 0] * op[:, 0] + op[:, 1] * op[:, 1]).astype(f) + op[:, 2] * op[:, 2]).astype(f)
    det = (((b * b).astype(f) - oo).astype(f) + (r * r).astype(f)).astype(f)
    ok = det >= 0
    t1 = (b[ok] - np.sqrt(det[ok]).astype(f)).astype(f)
    P = o[ok].astype(np.float64) + t1[:, None].astype(np.float64) * d[ok].astype(np.float64)
    C = c[ok].astype(np.float64)
    R = r[ok].astype(np.float64)
    off = np.abs(np.linalg.norm(P - C, axis=1) - R)
    scale = np.maximum(np.linalg.norm(C - o[ok].astype(np.float64), axis=1), R)
    assert ok.sum() > n // 4
    assert (off / scale).max() < 1.04e-3 < (1 / 128) / 3
