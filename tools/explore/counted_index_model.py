"""Driver of tools/explore/counted_index_model.cpp (build it to /tmp/libcim.so first, see its header):
first-bounce shadow rays of the configs[4] frame (camera ray -> nearest hit -> a random point of the
light sphere), work per counted shadow query of the current walk and of an index-ordered tree."""
import ctypes as C, sys, os, numpy as np, subprocess
sys.path.insert(0, 'se-195-project-ray-tracer_amd')
import rtamd
subprocess.run(["make", "-s", "-C", "tests/native", "libspt_bvh_check.so"], check=True)
L = C.CDLL("tests/native/libspt_bvh_check.so")
P = C.c_void_p
L.spt_bvh_wide_check.restype = C.c_longlong
L.spt_bvh_wide_check.argtypes = [P, C.c_int, P, P, C.c_longlong, P, P, P, P, P]
L.spt_bvh_walk_stats.argtypes = [P]
M = C.CDLL("/tmp/libcim.so")
M.cim_run.restype = C.c_longlong
M.cim_run.argtypes = [P, C.c_int, P, P, C.c_longlong, C.c_int, C.c_int, P]
S, n, cam = rtamd.scenes.complex10k()
W, H = 1920, 1080
rtamd.scenes.update_camera(cam, W, H)
rng = np.random.default_rng(1)
nr = 20000
px = rng.uniform(0, W, nr); py = rng.uniform(0, H, nr)
cx = np.array([cam.x.x, cam.x.y, cam.x.z], np.float32); cy = np.array([cam.y.x, cam.y.y, cam.y.z], np.float32)
cd = np.array([cam.dir.x, cam.dir.y, cam.dir.z], np.float32); co = np.array([cam.orig.x, cam.orig.y, cam.orig.z], np.float32)
d = (px / W - .5)[:, None] * cx + (py / H - .5)[:, None] * cy + cd
d /= np.linalg.norm(d, axis=1, keepdims=True)
o = np.tile(co, (nr, 1)) + 0.1 * d
rays = np.ascontiguousarray(np.concatenate([o, d], 1).astype(np.float32))
tw = np.zeros(nr, np.float32); ts = np.zeros(nr, np.float32); iw = np.zeros(nr, np.int32); is_ = np.zeros(nr, np.int32)
L.spt_bvh_wide_check(C.addressof(S), n, rays.ctypes.data, None, nr, tw.ctypes.data, iw.ctypes.data, ts.ctypes.data, is_.ctypes.data, None)
hitm = is_ >= 2                      # hit a fractal sphere or the ground (not the light)
hitm |= is_ == 1
hp = o[hitm] + ts[hitm, None] * d[hitm]
# shadow rays to a random point of the light sphere (centre (50,80,90), r 8)
m = hp.shape[0]
u = rng.normal(size=(m, 3)); u /= np.linalg.norm(u, axis=1, keepdims=True)
lp = np.array([50.0, 80.0, 90.0]) + 8.0 * u
sd = lp - hp; ln = np.linalg.norm(sd, axis=1); sd /= ln[:, None]
srays = np.ascontiguousarray(np.concatenate([hp, sd], 1).astype(np.float32))
maxt = (ln - 0.01).astype(np.float32)
v = C.c_longlong()
tw = np.zeros(m, np.float32); ts2 = np.zeros(m, np.float32); iw = np.zeros(m, np.int32); is2 = np.zeros(m, np.int32)
L.spt_bvh_walk_stats((C.c_longlong * 2)())
bad = L.spt_bvh_wide_check(C.addressof(S), n, srays.ctypes.data, maxt.ctypes.data, m, tw.ctypes.data, iw.ctypes.data, ts2.ctypes.data, is2.ctypes.data, C.addressof(v))
st = (C.c_longlong * 2)(); L.spt_bvh_walk_stats(st)
occ = (is2 >= 0).mean()
print("shadow rays %d, occluded %.2f; current counted walk: %.1f wide nodes, %.1f leaves, %.1f sphere tests per ray (bad %d)" % (m, occ, v.value / m, st[0] / m, st[1] / m, bad))
for leaf in (4, 8, 16):
    out = (C.c_longlong * 3)()
    M.cim_run(C.addressof(S), n, srays.ctypes.data, maxt.ctypes.data, m, leaf, 2, out)
    print("index-ordered binary tree, leaf %2d: %.1f binary nodes, %.1f sphere tests per ray (mismatch %d)" % (leaf, out[1] / m, out[2] / m, out[0]))
