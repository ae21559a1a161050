"""Host-side scene API mirroring the reference's object model.

Reference types (all by value in Zig) and their mirrors here:

* ``Texture`` union  (src/textures.zig:10-27): ``SolidColor``, ``CheckerTexture``,
  ``ImageTexture``, ``NoiseTexture`` (+ ``Perlin``, src/perlin.zig:76-101)
* ``Material`` union (src/material.zig:11-30): ``Lambertian``, ``Metal``,
  ``Dielectric``, ``DiffuseLight``, ``Isotropic``
* ``Sphere`` (src/objects.zig:68-149): ``Sphere.init`` / ``Sphere.initMoving``
* ``BVHTree`` (src/bvh.zig:17-104): ``BVHTree.init(objects, start, end)`` --
  flattens the objects to the C-ABI records (include/rtw_gpu.h) and hands them
  to ``rtw_scene_create``, which builds the reference-topology BVH natively
  and uploads it to the GPU.

Flattening order (one material per sphere, one texture per textured material,
Perlin tables and images de-duplicated by identity) is part of the fixture
contract checked in tests/test_scenes.py.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _abi
from .rng import DOMAIN_PERLIN, Stream, f32


def _v3(x) -> np.ndarray:
    a = np.asarray(x, dtype=np.float32).reshape(3)
    return a.copy()


# ---------------------------------------------------------------- textures
@dataclass(eq=False)
class Texture:
    kind: int


@dataclass(eq=False)
class SolidColor(Texture):
    color_value: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))

    @staticmethod
    def init(color) -> "SolidColor":
        return SolidColor(_abi.RTW_TEX_SOLID, _v3(color))


@dataclass(eq=False)
class CheckerTexture(Texture):
    inv_scale: np.float32 = f32(1)
    even: SolidColor = None
    odd: SolidColor = None

    @staticmethod
    def init(scale, even: SolidColor, odd: SolidColor) -> "CheckerTexture":
        """textures.zig:53-56: inv_scale = 1.0 / scale (f32)."""
        return CheckerTexture(_abi.RTW_TEX_CHECKER, f32(f32(1.0) / f32(scale)), even, odd)


@dataclass(eq=False)
class Image:
    """A decoded zstbi.Image: RGBA8 rows (src/rtw_image.zig, forced 4 components)."""
    rgba: np.ndarray  # (H, W, 4) uint8

    @property
    def width(self) -> int:
        return int(self.rgba.shape[1])

    @property
    def height(self) -> int:
        return int(self.rgba.shape[0])

    @staticmethod
    def load_npz(path: str, key: str = "rgba") -> "Image":
        with np.load(path, allow_pickle=False) as z:
            return Image(np.ascontiguousarray(z[key], dtype=np.uint8))


@dataclass(eq=False)
class ImageTexture(Texture):
    image: Image = None

    @staticmethod
    def init(images: Sequence[Image], image_index: int) -> "ImageTexture":
        return ImageTexture(_abi.RTW_TEX_IMAGE, images[image_index])


@dataclass(eq=False)
class Perlin:
    ranvec: np.ndarray  # (256, 3) f32
    perm_x: np.ndarray  # (256,) u16
    perm_y: np.ndarray
    perm_z: np.ndarray

    @staticmethod
    def init(seed: int = 0, table_id: int = 0) -> "Perlin":
        """perlin.zig:83-101 on the seeded stream (domain 3, a = table id).

        ``permute``'s randomIntRange(0, i) can return i + 1; at i = 255 the
        reference indexes p[256] (UB) -- clamped to 255 here."""
        s = Stream(seed, DOMAIN_PERLIN, table_id, 0)
        ranvec = np.zeros((256, 3), np.float32)
        for i in range(256):
            p = s.vec_range(-1, 1)
            ls = f32(f32(f32(p[0] * p[0]) + f32(p[1] * p[1])) + f32(p[2] * p[2]))
            ranvec[i] = p / np.sqrt(ls, dtype=np.float32)
        perms = []
        for _ in range(3):
            p = np.arange(256, dtype=np.uint16)
            for i in range(255, 0, -1):
                t = min(s.int_range(0, i), 255)
                p[i], p[t] = p[t], p[i]
            perms.append(p)
        return Perlin(ranvec, *perms)


@dataclass(eq=False)
class NoiseTexture(Texture):
    noise: Perlin = None
    scale: np.float32 = f32(1)

    @staticmethod
    def init(scale, perlin: Optional[Perlin] = None, seed: int = 0) -> "NoiseTexture":
        return NoiseTexture(_abi.RTW_TEX_NOISE, perlin if perlin is not None else Perlin.init(seed), f32(scale))


# ---------------------------------------------------------------- materials
@dataclass(eq=False)
class Material:
    kind: int
    texture: Optional[Texture] = None
    albedo: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    fuzz: np.float32 = f32(0)
    ir: np.float32 = f32(0)


class Lambertian:
    @staticmethod
    def init(texture: Texture) -> Material:
        return Material(_abi.RTW_MAT_LAMBERTIAN, texture)

    @staticmethod
    def fromColor(color) -> Material:
        return Material(_abi.RTW_MAT_LAMBERTIAN, SolidColor.init(color))


class Metal:
    @staticmethod
    def fromColor(color, f) -> Material:
        """material.zig:61-63: fuzz clamped to <= 1."""
        f = f32(f)
        return Material(_abi.RTW_MAT_METAL, None, _v3(color), f if f < f32(1) else f32(1))


class Dielectric:
    @staticmethod
    def init(ir) -> Material:
        return Material(_abi.RTW_MAT_DIELECTRIC, None, ir=f32(ir))


class DiffuseLight:
    @staticmethod
    def init(texture: Texture) -> Material:
        return Material(_abi.RTW_MAT_DIFFUSE_LIGHT, texture)

    @staticmethod
    def fromColor(color) -> Material:
        return Material(_abi.RTW_MAT_DIFFUSE_LIGHT, SolidColor.init(color))


class Isotropic:
    @staticmethod
    def init(texture: Texture) -> Material:
        return Material(_abi.RTW_MAT_ISOTROPIC, texture)

    @staticmethod
    def fromColor(color) -> Material:
        return Material(_abi.RTW_MAT_ISOTROPIC, SolidColor.init(color))


# ---------------------------------------------------------------- objects
@dataclass(eq=False)
class Sphere:
    center1: np.ndarray
    radius: np.float32
    mat: Material
    is_moving: bool = False
    center2: Optional[np.ndarray] = None

    @staticmethod
    def init(center1, radius, mat: Material) -> "Sphere":
        return Sphere(_v3(center1), f32(radius), mat)

    @staticmethod
    def initMoving(center1, center2, radius, mat: Material) -> "Sphere":
        return Sphere(_v3(center1), f32(radius), mat, True, _v3(center2))


@dataclass
class SceneArrays:
    """The neutral scene description handed across the C ABI."""
    spheres: np.ndarray
    materials: np.ndarray
    textures: np.ndarray
    perlins: np.ndarray
    images: List[Image]
    bvh_seed: int = 0
    bvh_mode: int = _abi.RTW_BVH_SAH   # or _abi.RTW_BVH_REFERENCE (bvh.zig topology, same closest hits)
    order_dir: tuple = (0.0, 0.0, 0.0)

    def desc(self):
        """Build an RtwSceneDesc (keeps the ctypes image array alive on self)."""
        imgs = (_abi.RtwImage * max(1, len(self.images)))()
        for i, im in enumerate(self.images):
            imgs[i].data = im.rgba.ctypes.data
            imgs[i].width = im.width
            imgs[i].height = im.height
            imgs[i].bytes_per_row = im.width * 4
        self._imgs = imgs
        d = _abi.RtwSceneDesc()
        d.spheres, d.n_spheres = _abi.ptr(self.spheres), len(self.spheres)
        d.materials, d.n_materials = _abi.ptr(self.materials), len(self.materials)
        d.textures, d.n_textures = _abi.ptr(self.textures), len(self.textures)
        d.images, d.n_images = (C.addressof(imgs) if self.images else 0), len(self.images)
        d.perlins, d.n_perlins = _abi.ptr(self.perlins), len(self.perlins)
        d.bvh_seed = self.bvh_seed
        d.bvh_mode = self.bvh_mode
        d.order_dir[:] = list(self.order_dir)
        return d


def flatten(objects: Sequence[Sphere], bvh_seed: int = 0, bvh_mode: Optional[int] = None) -> SceneArrays:
    """Objects -> C-ABI records.  bvh_mode: RTW_BVH_SAH (default, fastest) or
    RTW_BVH_REFERENCE (the reference's random-axis median tree, seeded by bvh_seed)."""
    sp = np.zeros(len(objects), _abi.SPHERE_DT)
    mats, texs, perlins, images = [], [], [], []

    def tex_index(t: Texture) -> int:
        rec = np.zeros((), _abi.TEXTURE_DT)
        rec["kind"] = t.kind
        if isinstance(t, SolidColor):
            rec["even"] = t.color_value
        elif isinstance(t, CheckerTexture):
            rec["scale"] = t.inv_scale
            rec["even"] = t.even.color_value
            rec["odd"] = t.odd.color_value
        elif isinstance(t, ImageTexture):
            idx = next((i for i, im in enumerate(images) if im is t.image), None)
            if idx is None:
                images.append(t.image)
                idx = len(images) - 1
            rec["image"] = idx
        elif isinstance(t, NoiseTexture):
            idx = next((i for i, p in enumerate(perlins) if p is t.noise), None)
            if idx is None:
                perlins.append(t.noise)
                idx = len(perlins) - 1
            rec["perlin"] = idx
            rec["scale"] = t.scale
        texs.append(rec)
        return len(texs) - 1

    for i, s in enumerate(objects):
        m = s.mat
        rec = np.zeros((), _abi.MATERIAL_DT)
        rec["kind"] = m.kind
        if m.texture is not None:
            rec["texture"] = tex_index(m.texture)
        rec["albedo"] = m.albedo
        rec["fuzz"] = m.fuzz
        rec["ir"] = m.ir
        mats.append(rec)
        sp[i]["center1"] = s.center1
        sp[i]["radius"] = s.radius
        if s.is_moving:
            sp[i]["center2"] = s.center2
            sp[i]["is_moving"] = 1
        sp[i]["material"] = len(mats) - 1
    pl = np.zeros(len(perlins), _abi.PERLIN_DT)
    for i, p in enumerate(perlins):
        pl[i]["ranvec"] = p.ranvec
        pl[i]["perm_x"], pl[i]["perm_y"], pl[i]["perm_z"] = p.perm_x, p.perm_y, p.perm_z
    return SceneArrays(sp, np.array(mats, _abi.MATERIAL_DT).reshape(-1),
                       np.array(texs, _abi.TEXTURE_DT).reshape(-1), pl, images, bvh_seed,
                       _abi.RTW_BVH_SAH if bvh_mode is None else bvh_mode)


def flatten_bvh(arrays: SceneArrays) -> np.ndarray:
    """Host-only BVH build + pre-order flatten (rtw_scene_flatten): the node array
    rtw_scene_create would upload."""
    L = _abi.lib()
    d = arrays.desc()
    n, depth = C.c_uint32(), C.c_uint32()
    _abi.check(L.rtw_scene_flatten(C.byref(d), None, 0, C.byref(n), C.byref(depth)), "rtw_scene_flatten")
    out = np.zeros(n.value, _abi.NODE_DT)
    _abi.check(L.rtw_scene_flatten(C.byref(d), out.ctypes.data, n.value, C.byref(n), C.byref(depth)),
               "rtw_scene_flatten")
    return out


class World:
    """A device-resident world: the result of ``BVHTree.init`` over the objects.

    Owns an ``rtw_ctx`` (one GPU).  ``Hittable{.tree = ...}`` in the reference."""

    def __init__(self, arrays: SceneArrays, device: int = 0):
        L = _abi.lib()
        self.arrays = arrays
        self.device = device
        self._desc = arrays.desc()
        h = C.c_void_p()
        _abi.check(L.rtw_scene_create(C.byref(self._desc), device, C.byref(h)), "rtw_scene_create")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None) and self.handle.value:
            _abi.lib().rtw_scene_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> dict:
        s = _abi.RtwSceneStats()
        _abi.check(_abi.lib().rtw_scene_stats_get(self.handle, C.byref(s)), "rtw_scene_stats_get")
        return {k: getattr(s, k) for k, _ in s._fields_ if not k.startswith("_")}

    def nodes(self) -> np.ndarray:
        n = C.c_uint32()
        _abi.check(_abi.lib().rtw_scene_nodes(self.handle, None, 0, C.byref(n)), "rtw_scene_nodes")
        out = np.zeros(n.value, _abi.NODE_DT)
        _abi.check(_abi.lib().rtw_scene_nodes(self.handle, out.ctypes.data, n.value, C.byref(n)), "rtw_scene_nodes")
        return out


class BVHTree:
    """bvh.zig:17-41 -- ``BVHTree.init(objects, start, end)`` returns a World."""

    @staticmethod
    def init(objects: Sequence[Sphere], start: int = 0, end: Optional[int] = None, seed: int = 0,
             device: int = 0, bvh_mode: Optional[int] = None) -> World:
        end = len(objects) if end is None else end
        return World(flatten(list(objects[start:end]), bvh_seed=seed, bvh_mode=bvh_mode), device)
