"""Regenerate the committed golden fixtures (run in the build container, where
/root/reference exists; the GPU box only reads the committed .npz files).

Fixtures (all data, no reference source):
  earthmap_rgba.npz  content/earthmap.jpg decoded by the reference's own vendored
                     stb_image v2.28 (oracle/_ref/stbi_decode, forced RGBA like
                     src/main.zig:1124); sha256 of the RGBA bytes is pinned.
  sky_rows.npz       top pure-sky rows of the reference's image2.ppm (400x225,
                     color.writeColor round(256*g)) and image.ppm (800x450,
                     stdout.zig floor(255.999*g)) -- the only reference-produced pixels.
  scenes.npz         book1 / ref_head scene records (seed 0) from the C oracle's
                     generator (src/main.zig:253-312 restated) + Perlin table 0.
  crops.npz          oracle float4 accumulators on fixed crops (see CROPS).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

REF = "/root/reference"
EARTH_SHA256 = "ba4d3b82533fdacb6fa6c44a0865d6af75ea3cc13f838d2561a6bddfefc32c5a"

# (name, scene, camera kwargs, crop (x0, y0, w, h), spp, seed)
BOOK1_CAM = dict(aspect_ratio=1.5, image_width=1200, samples_per_pixel=500, max_depth=50, background_mode=1)
CROPS = [
    ("book1_c2_center", "book1", BOOK1_CAM, (568, 368, 64, 64), 16, 0),
    ("book1_c2_ground", "book1", BOOK1_CAM, (100, 700, 64, 64), 16, 0),
    ("book1_c2_glass", "book1", BOOK1_CAM, (580, 300, 32, 32), 32, 7),
    ("head_small", "ref_head", dict(aspect_ratio=16 / 9, image_width=320, samples_per_pixel=8, max_depth=50,
                                     background_mode=1), (0, 0, 320, 180), 8, 3),
]


def read_ppm(path: str) -> np.ndarray:
    toks = open(path, "rb").read().split()
    assert toks[0] == b"P3"
    w, h, _mx = int(toks[1]), int(toks[2]), int(toks[3])
    vals = np.array([int(t) for t in toks[4:4 + w * h * 3]], dtype=np.int32)
    return vals.reshape(h, w, 3)


def earth() -> np.ndarray:
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    raw = subprocess.check_output([os.path.join(REPO, "oracle", "_ref", "stbi_decode"),
                                   os.path.join(REF, "content", "earthmap.jpg")])
    nl = raw.index(b"\n")
    w, h = map(int, raw[:nl].split())
    data = raw[nl + 1:]
    assert hashlib.sha256(data).hexdigest() == EARTH_SHA256
    return np.frombuffer(data, np.uint8).reshape(h, w, 4)


def scene_arrays(name: str, images):
    variant = {"book1": 0, "ref_head": 1}[name]
    return O.gen_book1(0, variant)


def main():
    rgba = earth()
    np.savez_compressed(os.path.join(HERE, "earthmap_rgba.npz"), rgba=rgba)

    img2 = read_ppm(os.path.join(REF, "image2.ppm"))
    img1 = read_ppm(os.path.join(REF, "image.ppm"))
    np.savez_compressed(os.path.join(HERE, "sky_rows.npz"), image2_rows=img2[:15].astype(np.int16),
                        image_rows=img1[:30].astype(np.int16),
                        image2_mean=img2.reshape(-1, 3).mean(0), image_mean=img1.reshape(-1, 3).mean(0))

    # the first 400 bytes of the reference's two PPM files: header + pixel text format (data)
    import json
    heads = {n: open(os.path.join(REF, n), "rb").read(400).decode("ascii") for n in ("image2.ppm", "image.ppm")}
    with open(os.path.join(HERE, "ppm_heads.json"), "w") as f:
        json.dump(heads, f, indent=1)

    b_sp, b_mt, b_tx = O.gen_book1(0, 0)
    h_sp, h_mt, h_tx = O.gen_book1(0, 1)
    perlin = O.gen_perlin(0, 0)
    np.savez_compressed(os.path.join(HERE, "scenes.npz"), book1_spheres=b_sp.view(np.uint8),
                        book1_materials=b_mt.view(np.uint8), book1_textures=b_tx.view(np.uint8),
                        head_spheres=h_sp.view(np.uint8), head_materials=h_mt.view(np.uint8),
                        head_textures=h_tx.view(np.uint8), perlin0=perlin.view(np.uint8))

    crops = {}
    for name, scene, camkw, (x0, y0, w, h), spp, seed in CROPS:
        sp, mt, tx = (b_sp, b_mt, b_tx) if scene == "book1" else (h_sp, h_mt, h_tx)
        world = O.World(sp, mt, tx, images=[rgba] if scene == "ref_head" else [])
        cam = O.camera(**camkw)
        W = cam.image_width
        pix = np.array([(y0 + j) * W + (x0 + i) for j in range(h) for i in range(w)], np.uint32)
        crops[name] = world.render_pixels(cam, seed, pix, 0, spp, threads=os.cpu_count() or 1)
        crops[name + "_pix"] = pix
    np.savez_compressed(os.path.join(HERE, "crops.npz"), **crops)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
