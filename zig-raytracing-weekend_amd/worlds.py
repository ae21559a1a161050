"""Scene builders (src/main.zig:88-312) restated on the seeded scene stream,
plus the benchmark configurations of BASELINE.json.

Every builder returns the object list; ``BVHTree.init`` turns it into a GPU
world.  Draw order follows the Zig source exactly (struct-literal fields are
evaluated left to right), so a given seed always yields the same scene.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np

from .rng import DOMAIN_SCENE, Stream, f32
from .scene import (CheckerTexture, ConstantMedium, Dielectric, DiffuseLight, Image, ImageTexture, Lambertian,
                    Metal, NoiseTexture, Perlin, Quad, RotateY, SolidColor, Sphere, Translate, createBox)

_HERE = os.path.dirname(os.path.abspath(__file__))


def _length(v: np.ndarray) -> np.float32:
    ls = f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))
    return np.sqrt(ls, dtype=np.float32)


def generate_world(seed: int = 0, variant: str = "book1", images: Optional[Sequence[Image]] = None) -> List[Sphere]:
    """generateWorld (src/main.zig:253-312).

    variant "book1": static spheres, solid grey ground, brown (-4,1,0) sphere
    (the Book-1 cover, image.ppm / image2.ppm).  variant "ref_head": exactly
    HEAD -- checker ground (scale 0.32), moving diffuse spheres
    (initMoving, +U[0,0.5)^3), earth image texture on the (-4,1,0) sphere.
    """
    if variant not in ("book1", "ref_head"):
        raise ValueError(variant)
    head = variant == "ref_head"
    s = Stream(seed, DOMAIN_SCENE)
    objs: List[Sphere] = []
    if head:
        checker = CheckerTexture.init(0.32, SolidColor.init([0.2, 0.3, 0.1]), SolidColor.init([0.9, 0.9, 0.9]))
        ground = Lambertian.init(checker)
    else:
        ground = Lambertian.fromColor([0.5, 0.5, 0.5])
    objs.append(Sphere.init([0, -1000, 0], 1000, ground))
    ref = np.array([4, 0.2, 0], np.float32)
    for ai in range(-11, 11):
        for bi in range(-11, 11):
            a, b = f32(ai), f32(bi)
            choose_mat = s.float()
            cx = f32(a + f32(f32(0.9) * s.float()))
            cz = f32(b + f32(f32(0.9) * s.float()))
            center = np.array([cx, f32(f32(0.4) * choose_mat), cz], np.float32)
            if _length(center - ref) > f32(0.9):
                if choose_mat < f32(0.8):
                    albedo = s.vec() * s.vec()
                    mat = Lambertian.fromColor(albedo)
                    if head:
                        d = np.array([s.range(0, 0.5), s.range(0, 0.5), s.range(0, 0.5)], np.float32)
                        objs.append(Sphere.initMoving(center, center + d, f32(f32(0.4) * choose_mat), mat))
                    else:
                        objs.append(Sphere.init(center, f32(f32(0.4) * choose_mat), mat))
                elif choose_mat < f32(0.95):
                    albedo = s.vec_range(0.5, 1)
                    fuzz = s.range(0, 0.5)
                    objs.append(Sphere.init(center, f32(f32(0.5) * choose_mat), Metal.fromColor(albedo, fuzz)))
                else:
                    ir = s.range(1, 2)
                    objs.append(Sphere.init(center, f32(f32(0.3) * choose_mat), Dielectric.init(ir)))
    objs.append(Sphere.init([0, 1, 0], 1.0, Dielectric.init(1.5)))
    if head:
        if not images:
            images = [earth_image()]
        objs.append(Sphere.init([-4, 1, 0], 1.0, Lambertian.init(ImageTexture.init(images, 0))))
    else:
        objs.append(Sphere.init([-4, 1, 0], 1.0, Lambertian.fromColor([0.4, 0.2, 0.1])))
    objs.append(Sphere.init([4, 1, 0], 1.0, Metal.fromColor([0.7, 0.6, 0.5], 0.1)))
    return objs


def stress_world(n: int = 100_000, seed: int = 0) -> List[Sphere]:
    """BASELINE config 4: n random spheres on the Book-1 ground.

    Per sphere, in draw order: choose_mat, x = -50 + 100u, z = -50 + 100u,
    radius = 0.05 + 0.25u, y = radius; then the Book-1 material draws."""
    s = Stream(seed, DOMAIN_SCENE, 4, 0)
    objs: List[Sphere] = [Sphere.init([0, -1000, 0], 1000, Lambertian.fromColor([0.5, 0.5, 0.5]))]
    for _ in range(n):
        choose_mat = s.float()
        x = s.range(-50, 50)
        z = s.range(-50, 50)
        r = s.range(0.05, 0.3)
        center = np.array([x, r, z], np.float32)
        if choose_mat < f32(0.8):
            albedo = s.vec() * s.vec()
            objs.append(Sphere.init(center, r, Lambertian.fromColor(albedo)))
        elif choose_mat < f32(0.95):
            albedo = s.vec_range(0.5, 1)
            fuzz = s.range(0, 0.5)
            objs.append(Sphere.init(center, r, Metal.fromColor(albedo, fuzz)))
        else:
            objs.append(Sphere.init(center, r, Dielectric.init(s.range(1, 2))))
    objs.append(Sphere.init([0, 1, 0], 1.0, Dielectric.init(1.5)))
    objs.append(Sphere.init([-4, 1, 0], 1.0, Lambertian.fromColor([0.4, 0.2, 0.1])))
    objs.append(Sphere.init([4, 1, 0], 1.0, Metal.fromColor([0.7, 0.6, 0.5], 0.1)))
    return objs


def earth_image() -> Image:
    """content/earthmap.jpg decoded by the reference's stb_image v2.28 (forced RGBA),
    committed as tests/golden/earthmap_rgba.npz (sha256 pinned in the tests)."""
    path = os.path.join(os.path.dirname(_HERE), "tests", "golden", "earthmap_rgba.npz")
    return Image.load_npz(path)


def earth_world(images: Optional[Sequence[Image]] = None) -> List[Sphere]:
    """earthWorld (src/main.zig:88-99)."""
    images = images or [earth_image()]
    return [Sphere.init([0, 0, 0], 2, Lambertian.init(ImageTexture.init(images, 0)))]


def two_spheres_world() -> List[Sphere]:
    """twoSpheresWorld (src/main.zig:101-113)."""
    checker = CheckerTexture.init(0.8, SolidColor.init([0.2, 0.3, 0.1]), SolidColor.init([0.9, 0.9, 0.9]))
    mat = Lambertian.init(checker)
    return [Sphere.init([0, -10, 0], 10, mat), Sphere.init([0, 10, 0], 10, mat)]


def two_perlin_world(seed: int = 0) -> List[Sphere]:
    """twoPerlinWorld (src/main.zig:115-125): one NoiseTexture(scale 4) shared by both spheres."""
    mat = Lambertian.init(NoiseTexture.init(4, Perlin.init(seed, 0)))
    return [Sphere.init([0, -1000, 0], 1000, mat), Sphere.init([0, 2, 0], 2, mat)]


def earth_perlin_world(seed: int = 0, images: Optional[Sequence[Image]] = None) -> List[Sphere]:
    """BASELINE config 5: earthmap image-textured sphere + Perlin-noise spheres
    (earthWorld + twoPerlinWorld, src/main.zig:88-125), placed side by side."""
    images = images or [earth_image()]
    noise = Lambertian.init(NoiseTexture.init(4, Perlin.init(seed, 0)))
    return [
        Sphere.init([0, -1000, 0], 1000, noise),
        Sphere.init([0, 2, 2.5], 2, noise),
        Sphere.init([0, 2, -2.5], 2, Lambertian.init(ImageTexture.init(images, 0))),
    ]


def quads_world() -> list:
    """quadsWorld (src/main.zig:127-144): five coloured quads."""
    left_red = Lambertian.init(SolidColor.init([1, 0.2, 0.2]))
    back_green = Lambertian.init(SolidColor.init([0.2, 1.0, 0.2]))
    right_blue = Lambertian.init(SolidColor.init([0.2, 0.2, 1.0]))
    upper_orange = Lambertian.init(SolidColor.init([1.0, 0.5, 0]))
    lower_teal = Lambertian.init(SolidColor.init([0.2, 0.8, 0.8]))
    return [
        Quad.init([-3, -2, 5], [0, 0, -4], [0, 4, 0], left_red),
        Quad.init([-2, -2, 0], [4, 0, 0], [0, 4, 0], back_green),
        Quad.init([3, -2, 1], [0, 0, 4], [0, 4, 0], right_blue),
        Quad.init([-2, -3, 1], [4, 0, 0], [0, 0, 4], upper_orange),
        Quad.init([-2, -3, 5], [4, 0, 0], [0, 0, -4], lower_teal),
    ]


def simple_light_world(seed: int = 0) -> list:
    """simpleLightWorld (src/main.zig:146-166): Perlin spheres lit by a quad and a sphere light
    (camera: camera.simple_light_camera)."""
    mat = Lambertian.init(NoiseTexture.init(4, Perlin.init(seed, 0)))
    difflight = DiffuseLight.init(SolidColor.init([4, 4, 4]))
    return [
        Sphere.init([0, -1000, 0], 1000, mat),
        Sphere.init([0, 2, 0], 2, mat),
        Quad.init([3, 1, -2], [2, 0, 0], [0, 2, 0], difflight),
        Sphere.init([0, 7, 0], 2, difflight),
    ]


def _cornell_walls(light_q, light_u, light_v, light_color):
    red = Lambertian.init(SolidColor.init([0.65, 0.05, 0.05]))
    white = Lambertian.init(SolidColor.init([0.73, 0.73, 0.73]))
    green = Lambertian.init(SolidColor.init([0.12, 0.45, 0.15]))
    light = DiffuseLight.init(SolidColor.init(light_color))
    walls = [
        Quad.init([555, 0, 0], [0, 555, 0], [0, 0, 555], green),
        Quad.init([0, 0, 0], [0, 555, 0], [0, 0, 555], red),
        Quad.init(light_q, light_u, light_v, light),
        Quad.init([0, 0, 0], [555, 0, 0], [0, 0, 555], white),
        Quad.init([555, 555, 555], [-555, 0, 0], [0, 0, -555], white),
        Quad.init([0, 0, 555], [555, 0, 0], [0, 555, 0], white),
    ]
    return walls, white


def cornell_box() -> list:
    """cornellBox (src/main.zig:168-205), HEAD's default scene (camera: camera.cornell_camera)."""
    objs, white = _cornell_walls([343, 554, 332], [-130, 0, 0], [0, 0, -105], [15, 15, 15])
    box1 = createBox([0, 0, 0], [165, 330, 165], white)
    box1 = RotateY.init(box1, 15)
    box1 = Translate.init(box1, [265, 0, 295])
    objs.append(box1)
    box2 = createBox([0, 0, 0], [165, 165, 165], white)
    box2 = RotateY.init(box2, -18)
    box2 = Translate.init(box2, [130, 0, 65])
    objs.append(box2)
    return objs


def cornell_smoke() -> list:
    """cornellBoxSmoke (src/main.zig:207-251): the two boxes as ConstantMedium (density 0.01),
    black and white smoke (camera: camera.cornell_smoke_camera)."""
    objs, white = _cornell_walls([113, 554, 127], [330, 0, 0], [0, 0, 305], [7, 7, 7])
    box1 = Translate.init(RotateY.init(createBox([0, 0, 0], [165, 330, 165], white), 15), [265, 0, 295])
    objs.append(ConstantMedium.initFromColor(box1, 0.01, [0, 0, 0]))
    box2 = Translate.init(RotateY.init(createBox([0, 0, 0], [165, 165, 165], white), -18), [130, 0, 65])
    objs.append(ConstantMedium.initFromColor(box2, 0.01, [1, 1, 1]))
    return objs

