"""Host-side scene API mirroring the reference's object model.

Reference types (all by value in Zig) and their mirrors here:

* ``Texture`` union  (src/textures.zig:10-27): ``SolidColor``, ``CheckerTexture``,
  ``ImageTexture``, ``NoiseTexture`` (+ ``Perlin``, src/perlin.zig:76-101)
* ``Material`` union (src/material.zig:11-30): ``Lambertian``, ``Metal``,
  ``Dielectric``, ``DiffuseLight``, ``Isotropic``
* ``Sphere`` (src/objects.zig:68-149): ``Sphere.init`` / ``Sphere.initMoving``
* ``Quad`` (src/objects.zig:193-262), ``HittableList`` (:264-290), ``Translate``
  (:292-331), ``RotateY`` (:333-443), ``ConstantMedium`` (:445-508) and
  ``createBox`` (:510-532)
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


@dataclass(eq=False)
class Quad:
    """Quad.init (objects.zig:201-210); the library derives normal, d, w and the box."""
    q: np.ndarray
    u: np.ndarray
    v: np.ndarray
    mat: Material

    @staticmethod
    def init(q, u, v, mat: Material) -> "Quad":
        return Quad(_v3(q), _v3(u), _v3(v), mat)


@dataclass(eq=False)
class HittableList:
    """objects.zig:264-290 (members: Spheres / Quads)."""
    objects: list = field(default_factory=list)

    @staticmethod
    def init() -> "HittableList":
        return HittableList([])

    def add(self, obj) -> None:
        self.objects.append(obj)


@dataclass(eq=False)
class Translate:
    """objects.zig:292-331."""
    object: object
    offset: np.ndarray

    @staticmethod
    def init(obj, offset) -> "Translate":
        return Translate(obj, _v3(offset))


@dataclass(eq=False)
class RotateY:
    """objects.zig:333-443 (sin/cos of degreesToRadians(angle), computed by the library)."""
    object: object
    angle: np.float32

    @staticmethod
    def init(obj, angle) -> "RotateY":
        return RotateY(obj, f32(angle))


@dataclass(eq=False)
class ConstantMedium:
    """objects.zig:445-508: boundary + density + Isotropic phase function."""
    boundary: object
    density: np.float32
    phase: Material

    @staticmethod
    def initFromColor(boundary, density, color) -> "ConstantMedium":
        return ConstantMedium(boundary, f32(density), Isotropic.init(SolidColor.init(color)))

    @staticmethod
    def initFromTexture(boundary, density, texture: Texture) -> "ConstantMedium":
        return ConstantMedium(boundary, f32(density), Isotropic.init(texture))


def createBox(a, b, mat: Material) -> HittableList:
    """objects.zig:510-532: the six sides of the box with opposite vertices a, b."""
    a, b = _v3(a), _v3(b)
    mn = np.minimum(a, b)
    mx = np.maximum(a, b)
    z = np.float32(0)
    dx = np.array([mx[0] - mn[0], z, z], np.float32)
    dy = np.array([z, mx[1] - mn[1], z], np.float32)
    dz = np.array([z, z, mx[2] - mn[2]], np.float32)
    sides = HittableList.init()
    sides.add(Quad.init([mn[0], mn[1], mn[2]], dx, dy, mat))
    sides.add(Quad.init([mx[0], mn[1], mx[2]], -dz, dy, mat))
    sides.add(Quad.init([mx[0], mn[1], mn[2]], -dx, dy, mat))
    sides.add(Quad.init([mn[0], mn[1], mn[2]], dz, dy, mat))
    sides.add(Quad.init([mn[0], mx[1], mx[2]], dx, -dz, mat))
    sides.add(Quad.init([mn[0], mn[1], mn[2]], dx, dz, mat))
    return sides


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
    quads: np.ndarray = field(default_factory=lambda: np.zeros(0, _abi.QUAD_DT))
    members: np.ndarray = field(default_factory=lambda: np.zeros(0, _abi.OBJECT_DT))
    instances: np.ndarray = field(default_factory=lambda: np.zeros(0, _abi.INSTANCE_DT))
    media: np.ndarray = field(default_factory=lambda: np.zeros(0, _abi.MEDIUM_DT))
    objects: Optional[np.ndarray] = None   # world_objects order; None = every sphere in order

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
        d.quads, d.n_quads = _abi.ptr(self.quads), len(self.quads)
        d.members, d.n_members = _abi.ptr(self.members), len(self.members)
        d.instances, d.n_instances = _abi.ptr(self.instances), len(self.instances)
        d.media, d.n_media = _abi.ptr(self.media), len(self.media)
        if self.objects is not None:
            d.objects, d.n_objects = _abi.ptr(self.objects), len(self.objects)
        return d


def flatten(objects: Sequence, bvh_seed: int = 0, bvh_mode: Optional[int] = None) -> SceneArrays:
    """world_objects -> C-ABI records.  bvh_mode: RTW_BVH_SAH (default, fastest) or
    RTW_BVH_REFERENCE (the reference's random-axis median tree, seeded by bvh_seed).

    Every primitive gets its own material record (and textured materials their own
    texture record), in object order; Perlin tables and images are shared by identity.
    Translate/RotateY chains over a HittableList (or one primitive) become an
    instance; a ConstantMedium's boundary is a sphere, quad or instance record that
    is not itself a world object."""
    spheres, quads, members, instances, media, objs = [], [], [], [], [], []
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

    def mat_index(m: Material) -> int:
        rec = np.zeros((), _abi.MATERIAL_DT)
        rec["kind"] = m.kind
        if m.texture is not None:
            rec["texture"] = tex_index(m.texture)
        rec["albedo"] = m.albedo
        rec["fuzz"] = m.fuzz
        rec["ir"] = m.ir
        mats.append(rec)
        return len(mats) - 1

    def prim(o) -> tuple:
        if isinstance(o, Sphere):
            rec = np.zeros((), _abi.SPHERE_DT)
            rec["center1"] = o.center1
            rec["radius"] = o.radius
            if o.is_moving:
                rec["center2"] = o.center2
                rec["is_moving"] = 1
            rec["material"] = mat_index(o.mat)
            spheres.append(rec)
            return (_abi.RTW_OBJ_SPHERE, len(spheres) - 1)
        if isinstance(o, Quad):
            rec = np.zeros((), _abi.QUAD_DT)
            rec["q"], rec["u"], rec["v"] = o.q, o.u, o.v
            rec["material"] = mat_index(o.mat)
            quads.append(rec)
            return (_abi.RTW_OBJ_QUAD, len(quads) - 1)
        raise TypeError(f"not a primitive: {type(o).__name__}")

    def hittable(o) -> tuple:
        if isinstance(o, (Sphere, Quad)):
            return prim(o)
        if isinstance(o, (Translate, RotateY, HittableList)):
            xfs = []
            while isinstance(o, (Translate, RotateY)):   # outermost first
                if isinstance(o, Translate):
                    xfs.append((_abi.RTW_XF_TRANSLATE, o.offset))
                else:
                    xfs.append((_abi.RTW_XF_ROTATE_Y, np.array([o.angle, 0, 0], np.float32)))
                o = o.object
            if len(xfs) > _abi.RTW_MAX_XF:
                raise ValueError(f"at most {_abi.RTW_MAX_XF} transforms per instance")
            inner = o.objects if isinstance(o, HittableList) else [o]
            rec = np.zeros((), _abi.INSTANCE_DT)
            rec["first"] = len(members)
            refs = [prim(m) for m in inner]
            for k, i in refs:
                members.append(np.array((k, i), _abi.OBJECT_DT))
            rec["count"] = len(refs)
            rec["n_xf"] = len(xfs)
            rec["flags"] = _abi.RTW_INST_LIST if isinstance(o, HittableList) else 0
            for j, (k, v) in enumerate(reversed(xfs)):    # xf[0] = innermost
                rec["xf"][j]["kind"] = k
                rec["xf"][j]["v"] = v
            instances.append(rec)
            return (_abi.RTW_OBJ_INSTANCE, len(instances) - 1)
        if isinstance(o, ConstantMedium):
            rec = np.zeros((), _abi.MEDIUM_DT)
            k, i = hittable(o.boundary)
            rec["boundary"]["kind"], rec["boundary"]["index"] = k, i
            rec["density"] = o.density
            rec["material"] = mat_index(o.phase)
            media.append(rec)
            return (_abi.RTW_OBJ_MEDIUM, len(media) - 1)
        raise TypeError(f"unsupported hittable: {type(o).__name__}")

    for o in objects:
        objs.append(hittable(o))
    pl = np.zeros(len(perlins), _abi.PERLIN_DT)
    for i, p in enumerate(perlins):
        pl[i]["ranvec"] = p.ranvec
        pl[i]["perm_x"], pl[i]["perm_y"], pl[i]["perm_z"] = p.perm_x, p.perm_y, p.perm_z

    def arr(lst, dt):
        return np.array(lst, dt).reshape(-1) if lst else np.zeros(0, dt)

    only_spheres = all(k == _abi.RTW_OBJ_SPHERE and i == n for n, (k, i) in enumerate(objs)) and \
        len(objs) == len(spheres)
    return SceneArrays(arr(spheres, _abi.SPHERE_DT), arr(mats, _abi.MATERIAL_DT), arr(texs, _abi.TEXTURE_DT), pl,
                       images, bvh_seed, _abi.RTW_BVH_SAH if bvh_mode is None else bvh_mode,
                       quads=arr(quads, _abi.QUAD_DT), members=arr(members, _abi.OBJECT_DT),
                       instances=arr(instances, _abi.INSTANCE_DT), media=arr(media, _abi.MEDIUM_DT),
                       objects=None if only_spheres else arr(objs, _abi.OBJECT_DT))


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

    def __init__(self, arrays: SceneArrays, device: int = 0, tuning: Optional[dict] = None):
        """tuning: rtw_tuning fields to override (A/B measurement; every setting renders the same image)."""
        L = _abi.lib()
        self.arrays = arrays
        self.device = device
        self._desc = arrays.desc()
        h = C.c_void_p()
        if tuning:
            t = _abi.tuning(**tuning)
            _abi.check(L.rtw_scene_create_ex(C.byref(self._desc), device, C.byref(t), C.byref(h)), "rtw_scene_create_ex")
        else:
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
    def init(objects: Sequence, start: int = 0, end: Optional[int] = None, seed: int = 0,
             device: int = 0, bvh_mode: Optional[int] = None) -> World:
        end = len(objects) if end is None else end
        return World(flatten(list(objects[start:end]), bvh_seed=seed, bvh_mode=bvh_mode), device)
