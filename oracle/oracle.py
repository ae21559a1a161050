"""ctypes wrapper of liboracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline.  It does not import the product package; scenes cross
as the neutral wire records (48-B spheres, 32-B materials, 48-B textures,
4608-B Perlin tables, RGBA8 images) documented in include/rtw_gpu.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

SPHERE_DT = np.dtype([("center1", "<f4", 3), ("radius", "<f4"), ("center2", "<f4", 3), ("is_moving", "<u4"),
                      ("material", "<u4"), ("_pad", "<u4", 3)])
MATERIAL_DT = np.dtype([("kind", "<u4"), ("texture", "<u4"), ("fuzz", "<f4"), ("ir", "<f4"),
                        ("albedo", "<f4", 3), ("_pad", "<f4")])
TEXTURE_DT = np.dtype([("kind", "<u4"), ("image", "<u4"), ("perlin", "<u4"), ("scale", "<f4"),
                       ("even", "<f4", 3), ("_p0", "<f4"), ("odd", "<f4", 3), ("_p1", "<f4")])
PERLIN_DT = np.dtype([("ranvec", "<f4", (256, 3)), ("perm_x", "<u2", 256), ("perm_y", "<u2", 256),
                      ("perm_z", "<u2", 256)])
QUAD_DT = np.dtype([("q", "<f4", 3), ("material", "<u4"), ("u", "<f4", 3), ("_p0", "<u4"), ("v", "<f4", 3),
                    ("_p1", "<u4")])
OBJECT_DT = np.dtype([("kind", "<u4"), ("index", "<u4")])
INSTANCE_DT = np.dtype([("first", "<u4"), ("count", "<u4"), ("n_xf", "<u4"), ("flags", "<u4"),
                        ("xf", np.dtype([("kind", "<u4"), ("v", "<f4", 3)]), 3)])
MEDIUM_DT = np.dtype([("boundary", OBJECT_DT), ("density", "<f4"), ("material", "<u4")])

F3 = C.c_float * 3


class OImage(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32),
                ("bytes_per_row", C.c_uint32), ("_pad", C.c_uint32)]


class OSceneDesc(C.Structure):
    _fields_ = [("spheres", C.c_void_p), ("n_spheres", C.c_uint32), ("materials", C.c_void_p),
                ("n_materials", C.c_uint32), ("textures", C.c_void_p), ("n_textures", C.c_uint32),
                ("images", C.c_void_p), ("n_images", C.c_uint32), ("perlins", C.c_void_p),
                ("n_perlins", C.c_uint32), ("bvh_seed", C.c_uint64), ("bvh_mode", C.c_uint32),
                ("order_dir", C.c_float * 3), ("quads", C.c_void_p), ("n_quads", C.c_uint32),
                ("members", C.c_void_p), ("n_members", C.c_uint32), ("instances", C.c_void_p),
                ("n_instances", C.c_uint32), ("media", C.c_void_p), ("n_media", C.c_uint32),
                ("objects", C.c_void_p), ("n_objects", C.c_uint32)]


class OCameraParams(C.Structure):
    _fields_ = [("aspect_ratio", C.c_float), ("image_width", C.c_uint32), ("image_height", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32), ("background_mode", C.c_uint32),
                ("background", F3), ("vfov", C.c_float), ("lookfrom", F3), ("lookat", F3), ("vup", F3),
                ("defocus_angle", C.c_float), ("focus_dist", C.c_float), ("pixel_offset", C.c_uint32)]


class OCamera(C.Structure):
    _fields_ = [("image_width", C.c_uint32), ("image_height", C.c_uint32), ("size", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32), ("background_mode", C.c_uint32),
                ("pixel_offset", C.c_uint32), ("_pad", C.c_uint32),
                ("center", F3), ("pixel00_loc", F3), ("pixel_delta_u", F3), ("pixel_delta_v", F3),
                ("u", F3), ("v", F3), ("w", F3), ("defocus_disk_u", F3), ("defocus_disk_v", F3),
                ("defocus_angle", C.c_float), ("background", F3)]


_lib = None
_fp = C.POINTER(C.c_float)


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    if os.path.isdir("/root/reference/libs/zstbi/libs/stbi"):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        sig = {
            "oracle_mix64": (u64, [u64]),
            "oracle_rng_floats": (None, [u64, u64, u32, u32, u32, vp]),
            "oracle_rng_u64": (None, [u64, u64, u32, u32, u32, vp]),
            "oracle_path_floats": (None, [u64, u32, u32, u32, vp]),
            "oracle_aabb_hit": (C.c_int, [vp, vp, vp, C.c_float, C.c_float]),
            "oracle_sphere_uv": (None, [vp, vp]),
            "oracle_libm": (None, [C.c_int, vp, vp, vp, u64]),
            "oracle_pow": (C.c_float, [C.c_float, C.c_float]),
            "oracle_reflect": (None, [vp, vp, vp]),
            "oracle_refract": (None, [vp, vp, C.c_float, vp]),
            "oracle_reflectance": (C.c_float, [C.c_float, C.c_float]),
            "oracle_sphere_hit": (C.c_int, [vp, vp, vp, C.c_float, C.c_float, C.c_float, vp]),
            "oracle_texture_value": (None, [vp, u32, C.c_float, C.c_float, vp, vp]),
            "oracle_quad_hit": (C.c_int, [vp, vp, vp, C.c_float, C.c_float, vp]),
            "oracle_medium_draw": (C.c_float, [u64, u32]),
            "oracle_perlin_noise": (C.c_float, [vp, vp]),
            "oracle_perlin_turb": (C.c_float, [vp, vp, C.c_int]),
            "oracle_gamma2": (None, [vp, vp]),
            "oracle_gen_perlin": (C.c_int, [u64, u32, vp]),
            "oracle_gen_book1": (C.c_int, [u64, u32, vp, vp, vp, u32, vp]),
            "oracle_camera_init": (C.c_int, [vp, vp]),
            "oracle_world_create": (vp, [vp]),
            "oracle_world_destroy": (None, [vp]),
            "oracle_world_stats": (C.c_int, [vp, vp]),
            "oracle_world_dump": (C.c_int, [vp, vp, u32]),
            "oracle_render_task": (C.c_int, [vp, vp, u64, u32, u32, vp, vp]),
            "oracle_render_threads": (C.c_int, [vp, vp, u64, u32, vp, vp]),
            "oracle_render_pixels": (C.c_int, [vp, vp, u64, vp, u32, u32, u32, vp, u32]),
            "oracle_sample": (None, [vp, vp, u64, u32, u32, vp]),
            "oracle_counters_enable": (None, [C.c_int]),
            "oracle_counters_reset": (None, []),
            "oracle_counters_get": (None, [vp]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


# ---------------------------------------------------------------- camera
def camera(aspect_ratio=16.0 / 9.0, image_width=800, image_height=0, samples_per_pixel=100, max_depth=16,
           background=(0.0, 0.0, 0.0), background_mode=0, vfov=20.0, lookfrom=(13.0, 2.0, 3.0),
           lookat=(0.0, 0.0, 0.0), vup=(0.0, 1.0, 0.0), defocus_angle=0.6, focus_dist=10.0,
           pixel_offset=1) -> OCamera:
    """Camera.init (camera.zig:118-154) on the given Camera fields."""
    p = OCameraParams()
    p.aspect_ratio, p.image_width, p.image_height = aspect_ratio, image_width, image_height
    p.samples_per_pixel, p.max_depth, p.background_mode = samples_per_pixel, max_depth, background_mode
    p.background[:] = list(background)
    p.vfov = vfov
    p.lookfrom[:], p.lookat[:], p.vup[:] = list(lookfrom), list(lookat), list(vup)
    p.defocus_angle, p.focus_dist, p.pixel_offset = defocus_angle, focus_dist, pixel_offset
    c = OCamera()
    lib().oracle_camera_init(C.byref(p), C.byref(c))
    return c


# ---------------------------------------------------------------- world
class World:
    """A BVHTree (reference topology) over the wire-format world objects."""

    @staticmethod
    def from_arrays(a, bvh_seed: Optional[int] = None) -> "World":
        """From a product SceneArrays-like object (plain numpy records; no product import)."""
        return World(a.spheres, a.materials, a.textures, a.perlins, [im.rgba for im in a.images],
                     a.bvh_seed if bvh_seed is None else bvh_seed, a.quads, a.members, a.instances, a.media,
                     a.objects)

    def __init__(self, spheres: np.ndarray, materials: np.ndarray, textures: np.ndarray,
                 perlins: Optional[np.ndarray] = None, images: Sequence[np.ndarray] = (), bvh_seed: int = 0,
                 quads: Optional[np.ndarray] = None, members: Optional[np.ndarray] = None,
                 instances: Optional[np.ndarray] = None, media: Optional[np.ndarray] = None,
                 objects: Optional[np.ndarray] = None):
        def rec(a, dt):
            return np.ascontiguousarray(a if a is not None else np.zeros(0, dt)).view(dt)
        self.quads, self.members = rec(quads, QUAD_DT), rec(members, OBJECT_DT)
        self.instances, self.media = rec(instances, INSTANCE_DT), rec(media, MEDIUM_DT)
        self.objects = None if objects is None else rec(objects, OBJECT_DT)
        self.spheres = np.ascontiguousarray(spheres).view(SPHERE_DT)
        self.materials = np.ascontiguousarray(materials).view(MATERIAL_DT)
        self.textures = np.ascontiguousarray(textures).view(TEXTURE_DT)
        self.perlins = np.ascontiguousarray(perlins if perlins is not None else np.zeros(0, PERLIN_DT)).view(PERLIN_DT)
        self.images = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        self._imgs = (OImage * max(1, len(self.images)))()
        for i, im in enumerate(self.images):
            self._imgs[i].data = im.ctypes.data
            self._imgs[i].height, self._imgs[i].width = im.shape[0], im.shape[1]
            self._imgs[i].bytes_per_row = im.shape[1] * 4
        d = OSceneDesc()
        d.spheres, d.n_spheres = _p(self.spheres), len(self.spheres)
        d.materials, d.n_materials = _p(self.materials), len(self.materials)
        d.textures, d.n_textures = _p(self.textures), len(self.textures)
        d.images, d.n_images = (C.addressof(self._imgs) if self.images else 0), len(self.images)
        d.perlins, d.n_perlins = _p(self.perlins), len(self.perlins)
        d.bvh_seed = bvh_seed
        d.quads, d.n_quads = _p(self.quads), len(self.quads)
        d.members, d.n_members = _p(self.members), len(self.members)
        d.instances, d.n_instances = _p(self.instances), len(self.instances)
        d.media, d.n_media = _p(self.media), len(self.media)
        if self.objects is not None:
            d.objects, d.n_objects = _p(self.objects), len(self.objects)
        self.desc = d
        self.handle = lib().oracle_world_create(C.byref(d))
        if not self.handle:
            raise ValueError("oracle_world_create failed")

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().oracle_world_destroy(self.handle)
                self.handle = None
        except Exception:  # interpreter shutdown
            pass

    def stats(self):
        o = np.zeros(4, np.uint32)
        lib().oracle_world_stats(self.handle, _p(o))
        return {"nodes": int(o[0]), "leaves": int(o[1]), "depth": int(o[2]), "axis_draws": int(o[3])}

    def dump(self) -> np.ndarray:
        n = self.stats()["nodes"]
        out = np.zeros((n, 8), np.float32)
        lib().oracle_world_dump(self.handle, _p(out), n)
        return out

    # ------------------------------------------------------------ hot loop
    def render_pixels(self, cam: OCamera, seed: int, pixels: np.ndarray, spp_begin: int, spp_end: int,
                      threads: int = 1) -> np.ndarray:
        pix = np.ascontiguousarray(pixels, dtype=np.uint32)
        out = np.zeros((len(pix), 4), np.float32)
        lib().oracle_render_pixels(self.handle, C.byref(cam), seed, _p(pix), len(pix), spp_begin, spp_end,
                                   _p(out), threads)
        return out

    def render_threads(self, cam: OCamera, seed: int, threads: int = 8, texture: bool = True):
        """startRender + 8 x Camera.render (main.zig:314-326, camera.zig:93-116)."""
        buf = np.zeros((cam.size, 4), np.float32)
        buf[:, 3] = 1.0
        tex = np.zeros((cam.size, 4), np.uint8) if texture else None
        lib().oracle_render_threads(self.handle, C.byref(cam), seed, threads, _p(buf), _p(tex) if texture else None)
        return buf, tex

    def sample(self, cam: OCamera, seed: int, pixel: int, sample: int) -> np.ndarray:
        out = np.zeros(3, np.float32)
        lib().oracle_sample(self.handle, C.byref(cam), seed, pixel, sample, _p(out))
        return out


def gen_book1(seed: int = 0, variant: int = 0, cap: int = 1024):
    sp = np.zeros(cap, SPHERE_DT)
    mt = np.zeros(cap, MATERIAL_DT)
    tx = np.zeros(cap, TEXTURE_DT)
    counts = np.zeros(3, np.uint32)
    rc = lib().oracle_gen_book1(seed, variant, _p(sp), _p(mt), _p(tx), cap, _p(counts))
    if rc != 0:
        raise ValueError("oracle_gen_book1 overflow")
    return sp[:counts[0]].copy(), mt[:counts[1]].copy(), tx[:counts[2]].copy()


def gen_perlin(seed: int = 0, table_id: int = 0) -> np.ndarray:
    out = np.zeros(1, PERLIN_DT)
    lib().oracle_gen_perlin(seed, table_id, _p(out))
    return out


def rng_floats(seed: int, domain: int, a: int, b: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    lib().oracle_rng_floats(seed, domain, a, b, n, _p(out))
    return out


def path_floats(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    """Render-domain draws of path (pixel, sample): rtw_rng.h rtw_path_float."""
    out = np.zeros(n, np.float32)
    lib().oracle_path_floats(seed, pixel, sample, n, _p(out))
    return out


def rng_u64(seed: int, domain: int, a: int, b: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint64)
    lib().oracle_rng_u64(seed, domain, a, b, n, _p(out))
    return out


def gamma2(accum: np.ndarray) -> np.ndarray:
    acc = np.ascontiguousarray(accum, dtype=np.float32).reshape(-1, 4)
    out = np.zeros((len(acc), 4), np.uint8)
    for i in range(len(acc)):
        lib().oracle_gamma2(_p(acc[i]), _p(out[i]))
    return out


class counters:
    """Instrumentation context: rays, inner nodes, leaves, texels, noise evals, samples."""

    def __enter__(self):
        lib().oracle_counters_reset()
        lib().oracle_counters_enable(1)
        return self

    def __exit__(self, *exc):
        o = np.zeros(6, np.uint64)
        lib().oracle_counters_get(_p(o))
        lib().oracle_counters_enable(0)
        self.rays, self.nodes, self.leaves, self.texels, self.noise, self.samples = (int(x) for x in o)
        return False
