"""The five BASELINE.json configurations as concrete (world, camera) pairs."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List

from . import worlds
from .camera import Camera, book1_camera, cornell_camera, cornell_smoke_camera, earth_perlin_camera, simple_light_camera
from .scene import Sphere


@dataclass
class Config:
    name: str
    description: str
    objects: Callable[[], List[Sphere]]
    camera: Callable[[], Camera]
    n_gpus: int = 1


CONFIGS = {
    "c1": Config("c1", "Book-1 random spheres 400x225, 10 spp, depth 50 (CPU plumbing case)",
                 lambda: worlds.generate_world(0, "book1"),
                 lambda: book1_camera(image_width=400, aspect_ratio=16.0 / 9.0, spp=10, max_depth=50)),
    "c2": Config("c2", "Book-1 random spheres 1200x800, 500 spp, depth 50, 1xMI355X",
                 lambda: worlds.generate_world(0, "book1"),
                 lambda: book1_camera(image_width=1200, aspect_ratio=1.5, spp=500, max_depth=50)),
    "c3": Config("c3", "Book-1 random spheres 3840x2160, 1024 spp, 8xMI355X tile-sharded",
                 lambda: worlds.generate_world(0, "book1"),
                 lambda: book1_camera(image_width=3840, aspect_ratio=16.0 / 9.0, spp=1024, max_depth=50), n_gpus=8),
    "c4": Config("c4", "BVH stress: 100k random spheres, 1920x1080, 256 spp",
                 lambda: worlds.stress_world(100_000, 0),
                 lambda: book1_camera(image_width=1920, aspect_ratio=16.0 / 9.0, spp=256, max_depth=50)),
    "c5": Config("c5", "Textured: earthmap image sphere + Perlin noise spheres, 1920x1080, 512 spp",
                 lambda: worlds.earth_perlin_world(0),
                 lambda: earth_perlin_camera(image_width=1920, spp=512, max_depth=50)),
    # SURVEY §8f scenes (not BASELINE configs): HEAD's default scene and its smoke variant
    "cornell": Config("cornell", "Cornell box (HEAD default scene) 600x600, 200 spp, depth 200",
                      worlds.cornell_box, lambda: cornell_camera(600, 200, 200)),
    "cornell_smoke": Config("cornell_smoke", "Cornell box with two ConstantMedium boxes 600x600, 200 spp, depth 50",
                            worlds.cornell_smoke, lambda: cornell_smoke_camera(600, 200, 50)),
    "simple_light": Config("simple_light", "Perlin spheres + quad/sphere lights 800x450, 100 spp, depth 50",
                           lambda: worlds.simple_light_world(0), lambda: simple_light_camera(800, 100)),
}
