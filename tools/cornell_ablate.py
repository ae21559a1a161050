"""Where a Cornell ray's time goes: ns per traced ray for the Cornell box (HEAD's default
scene) as the reference builds it (two Translate(RotateY(createBox)) instances), with the
boxes' 12 quads placed in world space as top-level objects (no instance transform, each
quad culled by the BVH on its own), and with the boxes removed.  Timing only: the
variants are different scenes.  Usage: python tools/cornell_ablate.py [spp]
"""
import ctypes as C
import importlib
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("zig-raytracing-weekend_amd")
S = pkg.scene
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32


def world_quads(box, angle, offset):
    th = math.radians(angle)
    c, s = math.cos(th), math.sin(th)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float64)
    out = []
    for q in box.objects:
        out.append(S.Quad.init(R @ q.q + np.asarray(offset), R @ q.u, R @ q.v, q.mat))
    return out


def variant(name):
    objs = pkg.worlds.cornell_box()
    if name == "reference":
        return objs
    walls = objs[:-2]
    if name == "no_boxes":
        return walls
    white = objs[-1].object.object.objects[0].mat
    b1 = S.createBox([0, 0, 0], [165, 330, 165], white)
    b2 = S.createBox([0, 0, 0], [165, 165, 165], white)
    return walls + world_quads(b1, 15, [265, 0, 295]) + world_quads(b2, -18, [130, 0, 65])


cam = pkg.cornell_camera()
cam.samples_per_pixel = spp
cam.init()
for name in ("reference", "world_quads", "no_boxes"):
    world = pkg.World(pkg.flatten(variant(name)))
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")

    def run(counters):
        opts = pkg._abi.RtwRenderOpts(0, 0, counters, None)
        pkg._abi.check(pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0,
                                                   acc.data_ptr(), None, C.byref(opts)), "rtw_render_device")

    run(cnt.data_ptr())
    rays = int(cnt[pkg._abi.RTW_STAT_RAYS].item())
    run(None)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    run(None)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    print(json.dumps({"variant": name, "ms": round(ms, 2), "rays_per_sample": round(rays / (cam.size * spp), 3),
                      "ns_per_ray": round(ms * 1e6 / rays, 4), "Msamples_s": round(cam.size * spp / ms / 1e3, 1)}),
          flush=True)
    world.close()
