"""zig-raytracing-weekend_amd -- MI355X-native drop-in for the per-pixel sample
loop of dariooddenino/zig-raytracing-weekend (src/camera.zig:93-208).

Host API (mirrors the reference's Zig API names):
  scene:   SolidColor, CheckerTexture, ImageTexture, NoiseTexture, Perlin,
           Lambertian, Metal, Dielectric, DiffuseLight, Isotropic,
           Sphere.init / Sphere.initMoving, BVHTree.init -> World
  camera:  Camera (+ init, render(state, task)), SharedStateImageWriter, Task,
           RayTraceState, start_render
  worlds:  generate_world, earth_world, two_spheres_world, two_perlin_world,
           stress_world, earth_perlin_world
The hot path runs in librtw_gpu.so (include/rtw_gpu.h) on gfx950.
"""
from . import _abi, configs, distributed, output, rng, worlds  # noqa: F401
from ._abi import RtwError, lib  # noqa: F401
from .camera import (Camera, RayTraceState, SharedStateImageWriter, Task, book1_camera,  # noqa: F401
                     cornell_camera, cornell_smoke_camera, earth_perlin_camera, progressive_render,
                     simple_light_camera, start_render)
from .scene import (BVHTree, CheckerTexture, ConstantMedium, Dielectric, DiffuseLight,  # noqa: F401
                    HittableList, Image, ImageTexture, Isotropic, Lambertian, Metal, NoiseTexture, Perlin, Quad,
                    RotateY, SceneArrays, SolidColor, Sphere, Translate, World, createBox, flatten)
