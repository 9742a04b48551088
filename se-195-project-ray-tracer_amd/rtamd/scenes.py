"""Scene inputs of the two reference renderers, restated as data.

These are the reference's own host-side inputs (not part of the device path):
  * whitted_scene()  -- Scene_InitScene, raytracer3.0.06.no_rec.samp/scene.cpp:217-272
                        (Primitive_Create :55-83)
  * cornell()        -- CornellSpheres, smallptgpu-v1.6/scene.h:29-40
  * cornell_camera() -- mainCPU/mainGPU camera (smallptCPU.cpp:184-185,
                        smallptGPU.cpp:850-851) + UpdateCamera (displayfunc.cpp:182-195)
  * read_scene()     -- ReadScene .scn parser (displayfunc.cpp:120-180)
  * hypersphere()    -- scene_build_complex.pl generator (:3-60)
  * complex10k()     -- the 10k-sphere config (BASELINE configs[4])
  * queue_scene()    -- Raytracer3.2.03 create_scene (scene.c:48-97, CHOOSE_SCENE 0)
                        after raytracer.c:721-746's copy into Primitive_2
All float arithmetic is float32, in the reference's order.
"""
import math

import numpy as np

from ._lib import Camera, Float4, Primitive, QPrimitive, Sphere, Vec3

f32 = np.float32
SPHERE, PLANE = 1, 2
DIFF, SPEC, REFR = 0, 1, 2


def _prim(p, typ, cx, cy, cz, rd, r, g, b, refl, refr, rindex, diff, spec, light):
    """Primitive_Create (scene.cpp:55-83)."""
    C = [f32(v) for v in (cx, cy, cz, rd, r, g, b, refl, refr, rindex, diff, spec)]
    cx, cy, cz, rd, r, g, b, refl, refr, rindex, diff, spec = C
    sph = typ == SPHERE
    p.type = typ
    p.m_Light = 1 if light else 0
    p.m_Color = Vec3(r, g, b)
    p.m_Refl, p.m_Refr, p.m_RIndex, p.m_Diff, p.m_Spec = refl, refr, rindex, diff, spec
    p.m_Centre = Vec3(cx, cy, cz) if sph else Vec3(0, 0, 0)
    p.m_Radius = rd if sph else 0
    p.m_SqRadius = f32(rd * rd) if sph else 0
    p.m_RRadius = (f32(f32(1.0) / rd) if rd > 0 else 0) if sph else 0
    p.plane_D = 0 if sph else rd
    p.plane_N = Vec3(0, 0, 0) if sph else Vec3(cx, cy, cz)


_WHITTED = [  # scene.cpp:228-261 (type, centre/normal, radius/depth, colour, refl, refr, rIndex, diff, spec, light)
    (PLANE, 0.0, 0.75, 0.0, 4.4, 0.6, 0.6, 0.6, 0.0, 0.0, 0.0, 0.4, 1.8, False),
    (SPHERE, 0.0, 6.5, 22.0, 0.35, 0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 1.0, 1.0, True),
    (SPHERE, 3.4, -3.40, 23.0, 2.5, 0.08, 0.08, 0.08, 1.9, 1.0, 2.3, 0.0, 0.0, False),
    (SPHERE, -0.7, -4.90, 27.0, 1.0, 0.07, 0.17, 0.07, 0.1, 1.5, 2.3, 0.2, 0.8, False),
    (SPHERE, -3.4, -3.40, 29.0, 2.5, 1.0, 1.0, 1.0, 0.8, 0.0, 0.0, 0.0, 0.0, False),
    (SPHERE, 0.5, -4.10, 29.0, 1.5, 1.5, 0.7, 0.7, 0.1, 0.0, 0.0, 0.2, 0.2, False),
    (SPHERE, -6.0, -4.10, 32.0, 1.5, 0.7, 0.7, 1.7, 0.2, 0.0, 0.0, 0.2, 0.2, False),
    (SPHERE, -6.7, -4.90, 29.0, 1.0, 0.07, 0.17, 0.07, 0.1, 1.5, 2.3, 0.2, 0.8, False),
    (SPHERE, 6.4, -4.90, 18.0, 1.0, 0.18, 0.18, 0.18, 1.7, 1.0, 2.6, 1.8, 0.0, False),
    (PLANE, 0.7, 0.0, 0.0, 5.4, 1.0, 0.6, 0.6, 0.0, 0.0, 0.0, 0.8, 1.5, False),
    (PLANE, -0.7, 0.0, 0.0, 5.4, 0.7, 0.6, 1.0, 0.0, 0.0, 0.0, 0.8, 0.8, False),
    (PLANE, 0.0, -0.8, 0.0, 5.4, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 1.2, 0.8, False),
    (PLANE, 0.0, 0.0, -0.14, 5.4, 2.5, 2.5, 2.5, 0.0, 0.0, 0.0, 1.2, 0.8, False),
    (PLANE, 0.0, 0.0, 0.72, 5.4, 0.1, 0.1, 0.1, 0.0, 0.0, 0.0, 1.0, 1.0, False),
    (SPHERE, -3.0, 6.5, 22.0, 0.35, 0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 0.0, 1.8, True),
    (SPHERE, 3.0, 6.5, 22.0, 0.35, 0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 0.0, 1.8, True),
    (SPHERE, -5.8, -5.55, 31.0, 0.35, 1.15, 0.35, 0.35, 1.0, 1.0, 2.3, 0.0, 1.8, True),
]


def whitted_scene():
    """(Primitive array, count) equal to m_Scene after Scene_InitScene()."""
    prims = (Primitive * len(_WHITTED))()
    for p, row in zip(prims, _WHITTED):
        _prim(p, *row)
    return prims, len(_WHITTED)


_CORNELL = [  # scene.h:29-40 (WALL_RAD 1e4f)
    (1e4, (1e4 + 1.0, 40.8, 81.6), (0, 0, 0), (.75, .25, .25), DIFF),
    (1e4, (-1e4 + 99.0, 40.8, 81.6), (0, 0, 0), (.25, .25, .75), DIFF),
    (1e4, (50.0, 40.8, 1e4), (0, 0, 0), (.75, .75, .75), DIFF),
    (1e4, (50.0, 40.8, -1e4 + 270.0), (0, 0, 0), (0, 0, 0), DIFF),
    (1e4, (50.0, 1e4, 81.6), (0, 0, 0), (.75, .75, .75), DIFF),
    (1e4, (50.0, -1e4 + 81.6, 81.6), (0, 0, 0), (.75, .75, .75), DIFF),
    (16.5, (27.0, 16.5, 47.0), (0, 0, 0), (.9, .9, .9), SPEC),
    (16.5, (73.0, 16.5, 78.0), (0, 0, 0), (.9, .9, .9), REFR),
    (7.0, (50.0, 81.6 - 15.0, 81.6), (12, 12, 12), (0, 0, 0), DIFF),
]


def _sphere(s, rad, p, e, c, refl):
    s.rad = f32(rad)
    s.p, s.e, s.c = Vec3(*map(f32, p)), Vec3(*map(f32, e)), Vec3(*map(f32, c))
    s.refl = refl


def cornell():
    """(Sphere array, count) equal to CornellSpheres.  Sums such as
    WALL_RAD + 1.f are float32 sums in the reference."""
    arr = (Sphere * len(_CORNELL))()
    W = f32(1e4)
    pos = [(W + f32(1.0), f32(40.8), f32(81.6)), (-W + f32(99.0), f32(40.8), f32(81.6)),
           (f32(50.0), f32(40.8), W), (f32(50.0), f32(40.8), -W + f32(270.0)),
           (f32(50.0), W, f32(81.6)), (f32(50.0), -W + f32(81.6), f32(81.6)),
           (f32(27.0), f32(16.5), f32(47.0)), (f32(73.0), f32(16.5), f32(78.0)),
           (f32(50.0), f32(81.6) - f32(15.0), f32(81.6))]
    for s, row, p in zip(arr, _CORNELL, pos):
        _sphere(s, row[0], p, row[2], row[3], row[4])
    return arr, len(_CORNELL)


def _v(v):
    return np.array([v.x, v.y, v.z], dtype=f32)


def _norm(a):
    l = f32(1.0) / f32(np.sqrt(f32(a[0] * a[0] + a[1] * a[1]) + f32(a[2] * a[2])))
    return np.array([l * a[0], l * a[1], l * a[2]], dtype=f32)


def _cross(a, b):
    return np.array([f32(a[1] * b[2]) - f32(a[2] * b[1]), f32(a[2] * b[0]) - f32(a[0] * b[2]),
                     f32(a[0] * b[1]) - f32(a[1] * b[0])], dtype=f32)


def update_camera(cam, width, height, fov_deg=45.0):
    """UpdateCamera (displayfunc.cpp:182-195): fov = (M_PI/180.f)*45.f in
    double, narrowed; x scaled by width*fov/height (float).  fov_deg other
    than the reference's 45 is for tests (narrow views of far scenes)."""
    d = _norm(_v(cam.target) - _v(cam.orig))
    fov = f32((math.pi / float(f32(180.0))) * fov_deg)
    x = _norm(_cross(d, np.array([0, 1, 0], dtype=f32)))
    k = f32(f32(f32(width) * fov) / f32(height))
    x = np.array([k * x[0], k * x[1], k * x[2]], dtype=f32)
    y = _norm(_cross(x, d))
    y = np.array([fov * y[0], fov * y[1], fov * y[2]], dtype=f32)
    cam.dir, cam.x, cam.y = Vec3(*d), Vec3(*x), Vec3(*y)
    return cam


def cornell_camera(width, height):
    """vinit(camera.orig, 50.f, 45.f, 205.6f); vinit(camera.target, 50.f,
    45 - 0.042612f, 204.6) then UpdateCamera."""
    cam = Camera()
    cam.orig = Vec3(f32(50.0), f32(45.0), f32(205.6))
    cam.target = Vec3(f32(50.0), f32(45.0) - f32(0.042612), f32(204.6))
    return update_camera(cam, width, height)


def read_scene(path):
    """ReadScene (displayfunc.cpp:120-180): returns (Sphere array, count, Camera
    with orig/target set; call update_camera for the basis)."""
    with open(path) as f:
        toks = f.read().split()
    if toks[0] != "camera":
        raise ValueError("Failed to read 6 camera parameters")
    cam = Camera()
    cv = [f32(float(t)) for t in toks[1:7]]
    cam.orig, cam.target = Vec3(*cv[:3]), Vec3(*cv[3:])
    if toks[7] != "size":
        raise ValueError("Failed to read sphere count")
    n = int(toks[8])
    arr = (Sphere * n)()
    k = 9
    for i in range(n):
        if toks[k] != "sphere":
            raise ValueError("Failed to read sphere #%d" % i)
        v = toks[k + 1:k + 12]
        mat = int(v[10])
        if mat not in (0, 1, 2):
            raise ValueError("Failed to read material type for sphere #%d: %d" % (i, mat))
        fv = [float(t) for t in v[:10]]
        _sphere(arr[i], fv[0], fv[1:4], fv[4:7], fv[7:10], mat)
        k += 12
    return arr, n, cam


def hypersphere(max_depth=4.0):
    """scene_build_complex.pl (HyperSphere/PrintSphere): list of
    (rad, (x, y, z), (0, 0, 0), (col2, 0, col1), DIFF) in emission order."""
    out = []

    def emit(depth, x, y, z, rad):
        k = depth / max_depth
        out.append((rad, (x, y, z), (0.0, 0.0, 0.0), (0.75 * (1.0 - k), 0.0, 0.75 * k), DIFF))

    def rec(depth, x, y, z, rad, d):
        if depth > max_depth:
            return
        emit(depth, x, y, z, rad)
        nr = rad / 2.0
        if d != 0:
            rec(depth + 1.0, x - rad - nr, y, z, nr, 1)
        if d != 1:
            rec(depth + 1.0, x + rad + nr, y, z, nr, 0)
        if d != 2:
            rec(depth + 1.0, x, y - rad - nr, z, nr, 3)
        if d != 3:
            rec(depth + 1.0, x, y + rad + nr, z, nr, 2)
        if d != 4:
            rec(depth + 1.0, x, y, z - rad - nr, nr, 5)
        if d != 5:
            rec(depth + 1.0, x, y, z + rad + nr, nr, 4)

    rec(0.0, 0.0, 0.0, 0.0, 15.0, 2)
    return out


def complex10k(total=10000):
    """BASELINE configs[4]: scenes/complex.scn's light + ground
    (complex.scn:3-4) followed by the first total-2 HyperSphere spheres at
    maxDepth 6, with complex.scn's camera (:1)."""
    rows = [(8.0, (50.0, 80.0, 90.0), (25.0, 25.0, 25.0), (0.0, 0.0, 0.0), DIFF),
            (10000.0, (0.0, -10050.0, 0.0), (0.0, 0.0, 0.0), (0.75, 0.75, 0.75), DIFF)]
    rows += hypersphere(6.0)[:total - 2]
    arr = (Sphere * len(rows))()
    for s, r in zip(arr, rows):
        _sphere(s, *r)
    cam = Camera()
    cam.orig = Vec3(f32(20.0), f32(80.0), f32(150.0))
    cam.target = Vec3(f32(0.0), f32(15.0), f32(0.0))
    return arr, len(rows), cam


def seeds(width, height, seed=1):
    """AllocateBuffers' seed fill (smallptGPU.cpp:105-110): srand(seed), then
    2*width*height glibc rand() words clamped to >= 2 (spt_seed_fill)."""
    from ._lib import lib
    out = np.empty(2 * width * height, dtype=np.uint32)
    lib().spt_seed_fill(out.ctypes.data, out.size, seed)
    return out


# Raytracer3.2.03 scene.c:61-92 (CHOOSE_SCENE 0): kind, material (r, g, b, refl,
# refr, refr_index, diff, spec), is_light, normal / centre xyz, depth / radius.
_QUEUE = [
    ("P", (0.6, 0.6, 0.6, 0.0, 0.0, 0.0, 0.4, 1.8), False, (0.0, 0.75, 0.0), 4.4),
    ("S", (0.08, 0.08, 0.08, 0.2, 1.0, 1.4, 0.0, 0.0), False, (3.4, -3.4, 23.0), 2.5),
    ("S", (0.07, 0.17, 0.07, 0.1, 1.0, 1.2, 0.0, 0.0), False, (-0.7, -4.90, 27.0), 1.0),
    ("S", (1.0, 1.0, 1.0, 0.8, 0.0, 0.0, 0.0, 0.0), False, (-3.4, -3.4, 29.0), 2.5),
    ("S", (1.5, 0.7, 0.7, 0.1, 0.0, 0.0, 0.2, 0.2), False, (0.5, -4.1, 29.0), 1.5),
    ("S", (0.7, 0.7, 1.7, 0.2, 0.0, 0.0, 0.2, 0.2), False, (-6.0, -4.1, 32.0), 1.5),
    ("S", (0.07, 0.17, 0.07, 0.3, 1.0, 1.2, 0.2, 0.8), False, (-6.7, -4.90, 29.0), 1.0),
    ("S", (0.08, 0.08, 0.08, 0.7, 1.0, 1.3, 0.8, 0.0), False, (6.4, -4.9, 18.0), 1.0),
    ("P", (1.0, 0.6, 0.6, 0.0, 0.0, 0.0, 0.8, 1.5), False, (0.7, 0.0, 0.0), 5.4),
    ("P", (0.7, 0.6, 1.0, 0.0, 0.0, 0.0, 0.8, 0.8), False, (-0.7, 0.0, 0.0), 5.4),
    ("P", (1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 1.2, 0.8), False, (0.0, -0.8, 0.0), 5.4),
    ("P", (1.5, 1.5, 1.5, 0.0, 0.0, 0.0, 1.2, 0.8), False, (0.0, 0.0, -0.14), 5.4),
    ("P", (0.1, 0.1, 0.1, 0.0, 0.0, 0.0, 1.0, 1.0), False, (0.0, 0.0, 0.72), 5.4),
    ("S", (0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 0.0, 1.8), True, (0.0, 6.5, 22.0), 0.35),
    ("S", (0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 0.0, 1.8), True, (-3.0, 6.5, 22.0), 0.35),
    ("S", (0.85, 0.85, 0.85, 0.0, 0.0, 0.0, 0.0, 1.8), True, (3.0, 6.5, 22.0), 0.35),
]


def queue_scene():
    """create_scene + the Primitive -> Primitive_2 copy: 17 primitives, the
    last one memset's zero record (n_primitives = 17 with 16 created,
    scene.c:55) -- a PLANE of normal 0 that no ray hits but every shadow ray
    tests.  Fields the reference leaves uninitialised (a sphere's normal, a
    plane's centre, dummy_3, colour w) are 0 here; no computation reads them."""
    P = (QPrimitive * 64)()
    for k, (kind, m, light, v, d) in enumerate(_QUEUE):
        p = P[k]
        r, g, b, refl, refr, ri, diff, spec = [f32(x) for x in m]
        p.m_color = Float4(r, g, b, 0)
        p.m_refl, p.m_refr, p.m_refr_index, p.m_diff, p.m_spec = refl, refr, ri, diff, spec
        p.is_light = 1 if light else 0
        if kind == "P":
            p.type = 0
            p.normal = Float4(f32(v[0]), f32(v[1]), f32(v[2]), 0)
            p.depth = f32(d)
        else:
            rad = f32(d)
            p.type = 1
            p.center = Float4(f32(v[0]), f32(v[1]), f32(v[2]), 0)
            p.radius = rad
            p.sq_radius = f32(rad * rad)
            p.r_radius = f32(f32(1.0) / rad)
    return P, len(_QUEUE) + 1
