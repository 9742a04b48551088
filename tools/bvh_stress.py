"""Randomised stress of the sphere hierarchy's exactness (tools only, GPU):
random sphere clouds over several decades of scale and radius, a huge ground
sphere, lights, cameras inside the cloud and up to 10^4 extents away (where
the per-ray culling margin is widest in absolute terms); each frame is
rendered with the hierarchy and with the full scan (RT_SPT_NO_BVH) and
compared bit for bit (colours, seeds, pixels, work counters).

    N=60 python tools/bvh_stress.py
    REPEAT=3 N=60 python tools/bvh_stress.py   # learnt order: cooperative heavy tiles (small frames)
    RT_SPT_TUNE=coop_g=2 REPEAT=2 N=60 python tools/bvh_stress.py   # ... at two (or 4) lanes per pixel
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import numpy as np  # noqa: E402
import rtamd  # noqa: E402

W, H, SPP = 96, 72, 8
DIFF, SPEC, REFR = 0, 1, 2


def scene(rng):
    n = int(rng.integers(300, 3000))
    ext = 10.0 ** rng.uniform(-1, 3)                 # cloud half-extent
    rmin, rmax = sorted(10.0 ** rng.uniform(-4, 0, 2))
    S = (rtamd.Sphere * n)()
    rtamd.scenes._sphere(S[0], 1e4 * ext, (0.0, -1e4 * ext - ext, 0.0), (0, 0, 0), (0.7, 0.7, 0.7), DIFF)
    rtamd.scenes._sphere(S[1], 0.1 * ext, (0.0, 2.0 * ext, 0.0), (20, 20, 20), (0, 0, 0), DIFF)
    rtamd.scenes._sphere(S[2], 0.05 * ext, (ext, 0.5 * ext, -ext), (5, 3, 3), (0, 0, 0), DIFF)
    for i in range(3, n):
        r = ext * 10.0 ** rng.uniform(np.log10(rmin), np.log10(rmax))
        c = rng.uniform(-ext, ext, 3)
        refl = int(rng.choice([DIFF, DIFF, DIFF, SPEC, REFR]))
        rtamd.scenes._sphere(S[i], r, tuple(c), (0, 0, 0), tuple(rng.uniform(0.2, 0.9, 3)), refl)
    far = float(rng.choice([0.0, 3.0, 30.0, 300.0, 3000.0, 10000.0]))
    cam = rtamd.Camera()
    if far == 0.0:
        o = rng.uniform(-ext, ext, 3)
        fov = 45.0
    else:
        u = rng.standard_normal(3)
        u[1] = abs(u[1])
        o = far * ext * u / np.linalg.norm(u)
        fov = min(45.0, 45.0 * 2.0 / far)
    cam.orig = rtamd.Vec3(*[float(v) for v in o])
    cam.target = rtamd.Vec3(*[float(v) for v in rng.uniform(-0.3 * ext, 0.3 * ext, 3)])
    rtamd.scenes.update_camera(cam, W, H, fov_deg=fov)
    return S, n, cam, "n=%d ext=%.3g r=[%.2g,%.2g]x far=%g" % (n, ext, rmin, rmax, far)


def render(S, n, cam, mode, no_bvh, counted):
    if no_bvh:
        os.environ["RT_SPT_NO_BVH"] = "1"
    else:
        os.environ.pop("RT_SPT_NO_BVH", None)
    f = rtamd.SmallptFrame(W, H, spheres=S, nspheres=n, camera=cam, mode=mode)
    f.render(SPP, counters=counted)
    return f


def main():
    count = int(os.environ.get("N", "40"))
    rng = np.random.default_rng(int(os.environ.get("SEED", "2026")))
    bad = 0
    t0 = time.time()
    for k in range(count):
        S, n, cam, desc = scene(rng)
        mode = int(rng.integers(0, 2))
        ref = render(S, n, cam, mode, True, True)
        for counted in [True, False] * int(os.environ.get("REPEAT", "1")):
            f = render(S, n, cam, mode, False, counted)
            same = (np.array_equal(f.colors.view(np.uint32), ref.colors.view(np.uint32))
                    and np.array_equal(f.seeds, ref.seeds) and np.array_equal(f.pixels, ref.pixels)
                    and (not counted or f.counters == ref.counters))
            if not same:
                bad += 1
                print("MISMATCH scene %d (%s, mode %d, counted %s)" % (k, desc, mode, counted), flush=True)
        print("scene %d ok: %s" % (k, desc), flush=True)
    print("bvh_stress: %d scenes, %d mismatches, %.0f s" % (count, bad, time.time() - t0), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
