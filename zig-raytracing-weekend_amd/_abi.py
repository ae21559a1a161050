"""ctypes binding of include/rtw_gpu.h (librtw_gpu.so, built in-tree by build()).

This is the Python stand-in for the FFI a Zig host would get from
``@cImport(@cInclude("rtw_gpu.h"))``.  Loading fails loudly if
the HIP library has not been built: there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTW_LIB") or os.path.join(_HERE, "librtw_gpu.so")  # RTW_LIB: A/B builds only

RTW_OK, RTW_E_INVALID, RTW_E_HIP, RTW_E_OOM, RTW_E_CANCELLED, RTW_E_NODEVICE = 0, -1, -2, -3, -4, -5
RTW_MAT_LAMBERTIAN, RTW_MAT_METAL, RTW_MAT_DIELECTRIC, RTW_MAT_DIFFUSE_LIGHT, RTW_MAT_ISOTROPIC = range(5)
RTW_TEX_SOLID, RTW_TEX_CHECKER, RTW_TEX_IMAGE, RTW_TEX_NOISE = range(4)
RTW_BG_CONSTANT, RTW_BG_GRADIENT = 0, 1
RTW_BVH_REFERENCE, RTW_BVH_SAH = 0, 1
RTW_PPM_WRITECOLOR, RTW_PPM_STDOUT = 0, 1
RTW_RENDER_NO_SYNC = 1
RTW_RENDER_FRESH = 2
RTW_ROWS_BALANCED = 0x80000000  # rows_per_block flag: the left-over rows split evenly over the shards (ABI 7)
RTW_STAT_RAYS, RTW_STAT_NODES, RTW_STAT_LEAVES, RTW_STAT_SAMPLES, RTW_STAT_NAN, RTW_STAT_TAIL_RAYS = 0, 1, 2, 3, 4, 5
RTW_STAT_COUNT = 8
RTW_K_GEN, RTW_K_TRACE, RTW_K_SHADE, RTW_K_TAIL, RTW_K_REDUCE, RTW_K_MEGA, RTW_K_COUNT = 0, 1, 2, 3, 4, 5, 8
RTW_K_NAMES = ("gen", "trace", "shade", "tail", "reduce", "mega")
RTW_KERNEL_WAVEFRONT, RTW_KERNEL_PERSISTENT, RTW_KERNEL_SIMPLE = 0, 1, 2
RTW_LDS_NODES, RTW_LDS_CNODES, RTW_LDS_MATERIALS, RTW_LDS_SHADE = 1, 2, 4, 8
RTW_LDS_GEOMETRY, RTW_LDS_PERLIN, RTW_LDS_MEGA_NODES, RTW_LDS_ALL = 16, 32, 64, 127
RTW_FUSE_STEP, RTW_FUSE_TAIL_LDS, RTW_FUSE_GLOBAL = 1, 2, 4
RTW_DEAL_RUNS, RTW_DEAL_TAIL, RTW_DEAL_SMALL, RTW_DEAL_ITERS, RTW_DEAL_SINGLES16 = 1, 2, 8, 16, 32
RTW_DEAL_SMALL_SORT, RTW_DEAL_ALL = 128, 187
RTW_DEVICE_CPU = -1

# numpy record layouts == the C structs (asserted against sizeof in tests)
SPHERE_DT = np.dtype([("center1", "<f4", 3), ("radius", "<f4"), ("center2", "<f4", 3), ("is_moving", "<u4"),
                      ("material", "<u4"), ("_pad", "<u4", 3)])
MATERIAL_DT = np.dtype([("kind", "<u4"), ("texture", "<u4"), ("fuzz", "<f4"), ("ir", "<f4"),
                        ("albedo", "<f4", 3), ("_pad", "<f4")])
TEXTURE_DT = np.dtype([("kind", "<u4"), ("image", "<u4"), ("perlin", "<u4"), ("scale", "<f4"),
                       ("even", "<f4", 3), ("_p0", "<f4"), ("odd", "<f4", 3), ("_p1", "<f4")])
PERLIN_DT = np.dtype([("ranvec", "<f4", (256, 3)), ("perm_x", "<u2", 256), ("perm_y", "<u2", 256),
                      ("perm_z", "<u2", 256)])
NODE_DT = np.dtype([("a", "<f4", 4), ("b", "<f4", 4)])
QUAD_DT = np.dtype([("q", "<f4", 3), ("material", "<u4"), ("u", "<f4", 3), ("_p0", "<u4"), ("v", "<f4", 3),
                    ("_p1", "<u4")])
OBJECT_DT = np.dtype([("kind", "<u4"), ("index", "<u4")])
XF_DT = np.dtype([("kind", "<u4"), ("v", "<f4", 3)])
RTW_MAX_XF = 3
RTW_INST_LIST = 1
INSTANCE_DT = np.dtype([("first", "<u4"), ("count", "<u4"), ("n_xf", "<u4"), ("flags", "<u4"),
                        ("xf", XF_DT, RTW_MAX_XF)])
MEDIUM_DT = np.dtype([("boundary", OBJECT_DT), ("density", "<f4"), ("material", "<u4")])
assert QUAD_DT.itemsize == 48 and OBJECT_DT.itemsize == 8 and INSTANCE_DT.itemsize == 64 and MEDIUM_DT.itemsize == 16
RTW_OBJ_SPHERE, RTW_OBJ_QUAD, RTW_OBJ_INSTANCE, RTW_OBJ_MEDIUM = 0, 1, 2, 3
RTW_XF_TRANSLATE, RTW_XF_ROTATE_Y = 0, 1
assert SPHERE_DT.itemsize == 48 and MATERIAL_DT.itemsize == 32 and TEXTURE_DT.itemsize == 48
assert PERLIN_DT.itemsize == 4608 and NODE_DT.itemsize == 32


class RtwImage(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32),
                ("bytes_per_row", C.c_uint32), ("_pad", C.c_uint32)]


class RtwSceneDesc(C.Structure):
    _fields_ = [("spheres", C.c_void_p), ("n_spheres", C.c_uint32),
                ("materials", C.c_void_p), ("n_materials", C.c_uint32),
                ("textures", C.c_void_p), ("n_textures", C.c_uint32),
                ("images", C.c_void_p), ("n_images", C.c_uint32),
                ("perlins", C.c_void_p), ("n_perlins", C.c_uint32),
                ("bvh_seed", C.c_uint64), ("bvh_mode", C.c_uint32), ("order_dir", C.c_float * 3),
                ("quads", C.c_void_p), ("n_quads", C.c_uint32),
                ("members", C.c_void_p), ("n_members", C.c_uint32),
                ("instances", C.c_void_p), ("n_instances", C.c_uint32),
                ("media", C.c_void_p), ("n_media", C.c_uint32),
                ("objects", C.c_void_p), ("n_objects", C.c_uint32)]


F3 = C.c_float * 3


class RtwCameraParams(C.Structure):
    _fields_ = [("aspect_ratio", C.c_float), ("image_width", C.c_uint32), ("image_height", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32), ("background_mode", C.c_uint32),
                ("background", F3), ("vfov", C.c_float), ("lookfrom", F3), ("lookat", F3), ("vup", F3),
                ("defocus_angle", C.c_float), ("focus_dist", C.c_float), ("pixel_offset", C.c_uint32)]


class RtwCamera(C.Structure):
    _fields_ = [("image_width", C.c_uint32), ("image_height", C.c_uint32), ("size", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32), ("background_mode", C.c_uint32),
                ("pixel_offset", C.c_uint32), ("_pad", C.c_uint32),
                ("center", F3), ("pixel00_loc", F3), ("pixel_delta_u", F3), ("pixel_delta_v", F3),
                ("u", F3), ("v", F3), ("w", F3), ("defocus_disk_u", F3), ("defocus_disk_v", F3),
                ("defocus_angle", C.c_float), ("background", F3)]


class RtwKernelTiming(C.Structure):
    _fields_ = [("ms", C.c_float * 8), ("launches", C.c_uint32 * 8)]


PROGRESS_FN = C.CFUNCTYPE(C.c_int, C.c_uint64, C.c_uint64, C.c_void_p)


class RtwRenderOpts(C.Structure):
    # ABI 5: running (a Zig bool, RenderThread.running: 0 = stop), cancel (non-zero = stop), progress
    _fields_ = [("spp_batch", C.c_uint32), ("flags", C.c_uint32), ("counters", C.c_void_p),
                ("timing", C.POINTER(RtwKernelTiming)), ("running", C.c_void_p), ("cancel", C.c_void_p),
                ("progress", PROGRESS_FN), ("user", C.c_void_p)]


def render_opts(spp_batch: int = 0, flags: int = 0, counters=None, timing=None, running=None, cancel=None,
                progress=None) -> RtwRenderOpts:
    """rtw_render_opts.  running: a ctypes.c_uint8 (or c_bool) flag, 0 = stop (the reference's
    RenderThread.running); cancel: a ctypes.c_int32, non-zero = stop; progress(done, total) -> True stops.
    The returned struct keeps the callback alive (attribute _keep)."""
    o = RtwRenderOpts(spp_batch, flags, counters, C.pointer(timing) if timing is not None else None)
    if running is not None:
        o.running = C.addressof(running)
    if cancel is not None:
        o.cancel = C.addressof(cancel)
    if progress is not None:
        cb = PROGRESS_FN(lambda done, total, user: 1 if progress(done, total) else 0)
        o.progress = cb
        o._keep = cb
    return o


class RtwTuning(C.Structure):
    _fields_ = [("kernel", C.c_uint32), ("bvh_orders", C.c_uint32), ("sah_max_leaf", C.c_uint32),
                ("compact_nodes", C.c_uint32), ("fast_box", C.c_uint32), ("fast_reject", C.c_uint32),
                ("lds", C.c_uint32), ("fuse", C.c_uint32), ("wf_iters", C.c_uint32), ("mega_shade_min", C.c_uint32),
                ("mega_waves", C.c_uint32), ("mega_tile_order", C.c_uint32), ("cpu_threads", C.c_uint32),
                ("wide_walk", C.c_uint32), ("wf_paths", C.c_uint64),
                ("tile_lists", C.c_uint32), ("hoist", C.c_uint32), ("sort_iters", C.c_uint32),
                ("sort_bits", C.c_uint32),
                ("sort_iters_split", C.c_uint32), ("object_tree", C.c_uint32), ("clds_shape", C.c_uint32), ("deal", C.c_uint32)]


def tuning(**fields) -> RtwTuning:
    """rtw_tuning_defaults() with `fields` overridden (every setting renders the same image)."""
    t = RtwTuning()
    lib().rtw_tuning_defaults(C.byref(t))
    for k, v in fields.items():
        if not hasattr(t, k):
            raise KeyError(f"rtw_tuning has no field {k!r}")
        setattr(t, k, v)
    return t


class RtwSceneStats(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_leaves", C.c_uint32), ("n_inner", C.c_uint32), ("depth", C.c_uint32),
                ("device_bytes", C.c_uint64), ("axis_draws", C.c_uint32), ("n_hoisted", C.c_uint32),
                ("extent", C.c_float), ("box_pad", C.c_float)]


# every symbol include/rtw_gpu.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "rtw_version": (C.c_int, []),
    "rtw_build_id": (C.c_char_p, []),
    "rtw_debug_sphere_filter": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p]),
    "rtw_last_error": (C.c_char_p, []),
    "rtw_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rtw_camera_init": (C.c_int, [C.POINTER(RtwCameraParams), C.POINTER(RtwCamera)]),
    "rtw_scene_create": (C.c_int, [C.POINTER(RtwSceneDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "rtw_scene_destroy": (None, [C.c_void_p]),
    "rtw_tuning_defaults": (None, [C.POINTER(RtwTuning)]),
    "rtw_scene_create_ex": (C.c_int, [C.POINTER(RtwSceneDesc), C.c_int, C.POINTER(RtwTuning), C.POINTER(C.c_void_p)]),
    "rtw_render": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                             C.c_uint64, C.c_void_p, C.c_void_p, PROGRESS_FN, C.c_void_p]),
    "rtw_render_ex": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_uint64, C.c_void_p, C.POINTER(RtwRenderOpts)]),
    "rtw_render_rows": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_uint64, C.c_void_p, C.POINTER(RtwRenderOpts)]),
    "rtw_render_multi_ex": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint64, C.c_void_p, C.POINTER(RtwRenderOpts)]),
    "rtw_multi_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
    "rtw_render_device": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p, C.POINTER(RtwRenderOpts)]),
    "rtw_render_rows_device": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.POINTER(RtwRenderOpts)]),
    "rtw_shard_rows": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "rtw_shard_image_row": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "rtw_shard_image_row_h": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "rtw_multi_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_void_p)]),
    "rtw_multi_destroy": (None, [C.c_void_p]),
    "rtw_render_multi_device": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint64, C.c_void_p, C.c_void_p, C.POINTER(RtwRenderOpts)]),
    "rtw_render_multi": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                   C.c_void_p, C.c_void_p]),
    "rtw_texture_from_accum": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "rtw_texture_from_accum_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "rtw_encode_ppm": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t,
                                 C.POINTER(C.c_size_t)]),
    "rtw_encode_png": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t,
                                 C.POINTER(C.c_size_t)]),
    "rtw_count_samples": (C.c_float, [C.c_void_p, C.c_uint64]),
    "rtw_scene_hash": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "rtw_checkpoint_write": (C.c_int, [C.c_char_p, C.POINTER(RtwCamera), C.c_uint64, C.c_uint64, C.c_uint32,
                                       C.c_void_p]),
    "rtw_checkpoint_read": (C.c_int, [C.c_char_p, C.POINTER(RtwCamera), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_void_p, C.c_uint64]),
    "rtw_scene_flatten": (C.c_int, [C.POINTER(RtwSceneDesc), C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_uint32)]),
    "rtw_scene_stats_get": (C.c_int, [C.c_void_p, C.POINTER(RtwSceneStats)]),
    "rtw_scene_nodes": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "rtw_debug_rng": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
    "rtw_debug_sample": (C.c_int, [C.c_void_p, C.POINTER(RtwCamera), C.c_uint64, C.c_uint32, C.c_uint32,
                                   C.c_void_p]),
}

_lib = None


class RtwError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load librtw_gpu.so (raises if the HIP extension was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"librtw_gpu.so not built at {LIB_PATH}: run __graft_entry__.build() "
                              "(the product has no CPU fallback)")
        # torch (if present) must own the HIP runtime first: load it before us so the
        # soname libamdhip64.so.7 resolves to one runtime per process.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        # an A/B build of an earlier ABI (RTW_LIB=...) may lack the newest entry points: those stay
        # unbound there (AttributeError on use); the in-tree library must export every one
        # (tests/test_abi.py)
        optional = os.environ.get("RTW_LIB") is not None
        for name, (res, args) in SIGNATURES.items():
            if optional and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code: int, where: str) -> None:
    if code != RTW_OK:
        raise RtwError(code, where, lib().rtw_last_error().decode(errors="replace"))


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0
