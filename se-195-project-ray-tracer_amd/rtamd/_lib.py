"""Loader for librt_hip.so (include/rt_hip.h) and the reference struct layouts.

The shared library is built in-tree by ``make -C se-195-project-ray-tracer_amd``
(``__graft_entry__.build()``).  There is no CPU fallback: if the library or a
gfx950 device is missing, calls raise :class:`RTError`.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RT_HIP_LIB overrides the library path (A/B builds of kernel variants).
LIB_PATH = os.environ.get("RT_HIP_LIB") or os.path.join(PKG_DIR, "librt_hip.so")

RT_OK, RT_ERR_INVALID, RT_ERR_HIP, RT_ERR_NODEVICE = 0, -1, -2, -3
SPT_PATH_TRACING, SPT_DIRECT_LIGHTING = 0, 1
SPT_COUNT_RAYS = 0x100
SPT_COST_MAX = 0x200
SPT_LIST_SET = 0x800

# Every symbol include/rt_hip.h declares (checked by tests/test_abi.py).
EXPORTS = ("rt_last_error", "rt_device_count", "rt_set_device", "rt_release", "rt_cached_bytes",
           "rt_host_alloc", "rt_host_free",
           "rtw_render", "rtw_render_async", "rtw_render_ocl", "rtw_render_ocl_async", "spt_render", "spt_render_async", "spt_seed_fill",
           "spt_scene_create", "spt_scene_destroy", "spt_scene_release_captures", "spt_scene_render_async", "spt_scene_render_groups_async",
           "spt_group_count", "spt_scene_render_list_async", "spt_groups_pack_async", "spt_groups_unpack_async",
           "spt_pack_pixels_async",
           "spt_multi_create", "spt_multi_destroy", "spt_multi_set_scene", "spt_multi_bands", "spt_multi_upload",
           "spt_multi_render_async", "spt_multi_gather_async", "spt_multi_sync", "spt_multi_download",
           "spt_multi_read_frame", "spt_multi_counters", "spt_multi_band_buffers", "spt_render_multi",
           "spt_multi_cache_info", "rtq_render", "rtq_render_async")


class RTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (rt code %d)" % (msg, code))
        self.code = code


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Primitive(C.Structure):
    """raytracer3.0.06.no_rec.samp/raytracer.h:23-32 (96 bytes)."""
    _fields_ = [("type", C.c_int32), ("m_Light", C.c_int32), ("m_Centre", Vec3),
                ("m_SqRadius", C.c_float), ("m_Radius", C.c_float), ("m_RRadius", C.c_float),
                ("plane_N", Vec3), ("plane_D", C.c_float), ("plane_cell", C.c_float * 4),
                ("m_Color", Vec3), ("m_Refl", C.c_float), ("m_Refr", C.c_float),
                ("m_Diff", C.c_float), ("m_Spec", C.c_float), ("m_RIndex", C.c_float)]


class Sphere(C.Structure):
    """smallptgpu-v1.6/geom.h:43-47 (44 bytes)."""
    _fields_ = [("rad", C.c_float), ("p", Vec3), ("e", Vec3), ("c", Vec3), ("refl", C.c_int32)]


class Camera(C.Structure):
    """smallptgpu-v1.6/camera.h:29-34 (60 bytes)."""
    _fields_ = [("orig", Vec3), ("target", Vec3), ("dir", Vec3), ("x", Vec3), ("y", Vec3)]


class Float4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class QPrimitive(C.Structure):
    """Raytracer3.2.03 raytracer_non_OpenCL.c:67-81 Primitive_2 (96 bytes)."""
    _fields_ = [("m_color", Float4), ("m_refl", C.c_float), ("m_diff", C.c_float), ("m_refr", C.c_float),
                ("m_refr_index", C.c_float), ("m_spec", C.c_float), ("dummy_3", C.c_float),
                ("type", C.c_int32), ("is_light", C.c_uint8), ("pad_", C.c_uint8 * 3),
                ("normal", Float4), ("center", Float4), ("depth", C.c_float), ("radius", C.c_float),
                ("sq_radius", C.c_float), ("r_radius", C.c_float)]


assert C.sizeof(Primitive) == 96 and C.sizeof(Sphere) == 44 and C.sizeof(Camera) == 60
assert C.sizeof(QPrimitive) == 96

_lib = None


def lib():
    """The loaded librt_hip.so (raises RTError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RTError(RT_ERR_NODEVICE, "librt_hip.so not built (%s); run "
                      "`make -C se-195-project-ray-tracer_amd` or __graft_entry__.build()" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, i, u, u64p = C.c_void_p, C.c_int, C.c_uint, C.c_void_p
    L.rt_last_error.restype = C.c_char_p
    L.rt_device_count.restype = i
    L.rt_set_device.argtypes = [i]
    L.rt_cached_bytes.restype = C.c_size_t
    L.rt_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
    L.rt_host_free.argtypes = [C.c_void_p]
    L.rtw_render.argtypes = [vp, i, vp, i, i, i, i, u64p]
    L.rtw_render_async.argtypes = [vp, i, vp, i, i, i, i, u64p, vp]
    L.rtw_render_ocl.argtypes = [vp, i, vp, i, i, u64p]
    L.rtw_render_ocl_async.argtypes = [vp, i, vp, i, i, u64p, vp]
    L.spt_render.argtypes = [vp, u, vp, vp, vp, vp, i, i, i, i, i, u64p]
    L.spt_render_async.argtypes = [vp, u, vp, vp, vp, vp, vp, i, i, i, i, i, i, i, u64p, vp]
    L.spt_seed_fill.argtypes = [vp, C.c_size_t, u]
    L.spt_scene_create.argtypes = [vp, u, C.POINTER(vp)]
    L.spt_scene_destroy.argtypes = [vp]
    if hasattr(L, "spt_scene_release_captures"):
        L.spt_scene_release_captures.argtypes = [vp]
    L.spt_scene_render_async.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, i, i, i, i, u64p, vp]
    if hasattr(L, "spt_scene_render_groups_async"):
        L.spt_scene_render_groups_async.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, i, i, i, i, u64p, vp]
    if hasattr(L, "spt_pack_pixels_async"):   # (absent from older A/B builds under RT_HIP_LIB)
        L.spt_pack_pixels_async.argtypes = [vp, vp, i, i, i, i, vp]
    if hasattr(L, "spt_scene_render_list_async"):
        L.spt_group_count.argtypes = [i, i]
        L.spt_scene_render_list_async.argtypes = [vp, vp, vp, vp, vp, vp, i, i, vp, i, i, i, i, u64p, vp, vp]
        L.spt_groups_pack_async.argtypes = [vp, i, i, vp, i, vp, vp]
        L.spt_groups_unpack_async.argtypes = [vp, i, i, vp, i, vp, vp]
    L.spt_seed_fill.restype = None
    if hasattr(L, "spt_multi_create"):
        ip = C.POINTER(C.c_int)
        L.spt_multi_create.argtypes = [vp, u, i, i, vp, i, C.POINTER(vp)]
        L.spt_multi_destroy.argtypes = [vp]
        L.spt_multi_set_scene.argtypes = [vp, vp, u]
        L.spt_multi_bands.argtypes = [vp, vp]
        L.spt_multi_upload.argtypes = [vp, vp, vp]
        L.spt_multi_render_async.argtypes = [vp, vp, i, i, i, i]
        L.spt_multi_gather_async.argtypes = [vp]
        L.spt_multi_sync.argtypes = [vp]
        L.spt_multi_download.argtypes = [vp, vp, vp, vp]
        L.spt_multi_read_frame.argtypes = [vp, i, vp, vp]
        L.spt_multi_counters.argtypes = [vp, vp]
        L.spt_multi_band_buffers.argtypes = [vp, i, ip, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp),
                                             C.POINTER(vp)]
        L.spt_render_multi.argtypes = [vp, u, vp, vp, vp, vp, i, i, i, i, i, u64p, vp, i]
        if hasattr(L, "spt_multi_cache_info"):
            L.spt_multi_cache_info.argtypes = [vp]
    if hasattr(L, "rtq_render"):
        L.rtq_render.argtypes = [vp, i, vp, i, i, u64p]
        L.rtq_render_async.argtypes = [vp, i, vp, i, i, i, i, u64p, vp]
    _lib = L
    return L


def check(rc):
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RTError(rc, msg.decode() if msg else "rt error")
    return rc


def device_count():
    n = lib().rt_device_count()
    return max(n, 0)


def set_device(dev):
    check(lib().rt_set_device(int(dev)))
