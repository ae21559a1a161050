"""DIAGNOSTIC: object-scene parity triage on the GPU (match fraction per
kernel / BVH mode / slab test, and per-sample values of a few mismatching pixels)."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import torch  # noqa: E402,F401

rtw = importlib.import_module("zig-raytracing-weekend_amd")
import oracle as O  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "quads"
kw = dict(aspect_ratio=1.0, vfov=80.0, lookfrom=(0.0, 0.0, 9.0), lookat=(0.0, 0.0, 0.0), defocus_angle=0.0,
          background=(0.7, 0.8, 1.0)) if scene == "quads" else \
    dict(aspect_ratio=1.0, vfov=40.0, lookfrom=(278.0, 278.0, -800.0), lookat=(278.0, 278.0, 0.0), defocus_angle=0.0)
build = {"quads": rtw.worlds.quads_world, "cornell": rtw.worlds.cornell_box, "smoke": rtw.worlds.cornell_smoke}[scene]
W, spp, depth = 48, 1, int(sys.argv[2]) if len(sys.argv) > 2 else 50
for mode in (rtw._abi.RTW_BVH_REFERENCE, rtw._abi.RTW_BVH_SAH):
    arr = rtw.flatten(build(), bvh_mode=mode)
    ow = O.World.from_arrays(arr)
    ocam = O.camera(image_width=W, samples_per_pixel=spp, max_depth=depth, **kw)
    ref = ow.render_pixels(ocam, 3, np.arange(W * W, dtype=np.uint32), 0, spp)
    cam = rtw.Camera(image_width=W, samples_per_pixel=spp, max_depth=depth, **kw).init()
    for env in ({"RTW_KERNEL": "v0"}, {"RTW_KERNEL": "wf"}, {"RTW_KERNEL": "wf", "RTW_FASTBOX": "0"}):
        for k in ("RTW_KERNEL", "RTW_FASTBOX"):
            os.environ.pop(k, None)
        os.environ.update(env)
        world = rtw.World(arr)
        buf = np.zeros((cam.size, 4), np.float32)
        rtw._abi.check(rtw.lib().rtw_render(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 3,
                                            buf.ctypes.data, None, rtw._abi.PROGRESS_FN(0), None), "render")
        ok = (np.abs(buf[:, :3] - ref[:, :3]) <= 1e-4 * np.maximum(1, np.abs(ref[:, :3]))).all(axis=1)
        print("mode", mode, env, "match", ok.mean(), flush=True)
        bad = np.nonzero(~ok)[0][:4]
        for p in bad:
            out = np.zeros(3, np.float32)
            rtw.lib().rtw_debug_sample(world.handle, C.byref(cam.derived), 3, int(p), 0, out.ctypes.data)
            print("   pixel", p, "gpu", buf[p, :3], "dbg", out, "oracle", ref[p, :3], ow.sample(ocam, 3, int(p), 0))
        world.close()
