"""DIAGNOSTIC: image identity between node orderings (RTW_ORDERS=1 vs 8) on a config,
with oracle checks of mismatching samples."""
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

cfg = rtw.configs.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
arr = rtw.flatten(cfg.objects())
cam = cfg.camera()
cam.samples_per_pixel = 2
cam.init()
outs = {}
for o in ("1", "8"):
    os.environ["RTW_ORDERS"] = o
    w = rtw.World(arr)
    buf = np.zeros((cam.size, 4), np.float32)
    rtw._abi.check(rtw.lib().rtw_render(w.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0, buf.ctypes.data,
                                        None, rtw._abi.PROGRESS_FN(0), None), "render")
    outs[o] = (buf, w)
diff = np.nonzero((outs["1"][0] != outs["8"][0]).any(axis=1))[0]
print("pixels differing:", len(diff), "of", cam.size, flush=True)
if len(diff):
    ow = O.World.from_arrays(arr)
    d = cam.derived
    ocam = O.camera(aspect_ratio=cam.aspect_ratio, image_width=d.image_width, image_height=d.image_height,
                    samples_per_pixel=2, max_depth=d.max_depth, background=tuple(d.background),
                    background_mode=d.background_mode, vfov=cam.vfov, lookfrom=cam.lookfrom, lookat=cam.lookat,
                    vup=cam.vup, defocus_angle=cam.defocus_angle, focus_dist=cam.focus_dist)
    for p in diff[:6]:
        for s in range(2):
            o = ow.sample(ocam, 0, int(p), s)
            g = {}
            for k in ("1", "8"):
                out = np.zeros(3, np.float32)
                rtw.lib().rtw_debug_sample(outs[k][1].handle, C.byref(cam.derived), 0, int(p), s, out.ctypes.data)
                g[k] = out
            print(p, s, "oracle", o, "orders1", g["1"], "orders8", g["8"], flush=True)
