"""DIAGNOSTIC: C2's iteration 0 alone (max_depth 1: camera ray, first hit, shading, no survivors
stored) with and without the camera-ray tile lists, and at max_depth 2 (+ the survivors' stores
and one bounce)."""
import ctypes as C
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

pkg = importlib.import_module("zig-raytracing-weekend_amd")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cfg = pkg.configs.CONFIGS["c2"]
arr = pkg.flatten(cfg.objects())
for tl in (1, 0):
    world = pkg.World(arr, tuning={"tile_lists": tl})
    for depth in (1, 2):
        cam = cfg.camera()
        cam.samples_per_pixel = spp
        cam.max_depth = depth
        cam.init()
        acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
        for rep in range(3):
            t = pkg._abi.RtwKernelTiming()
            opts = pkg._abi.RtwRenderOpts(0, 0, None, C.pointer(t))
            pkg._abi.check(pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0,
                                                       acc.data_ptr(), None, C.byref(opts)), "render")
        print(f"tile_lists {tl} depth {depth}: " + " ".join(
            f"{n}={t.ms[i]:.2f}ms/{t.launches[i]}" for i, n in enumerate(pkg._abi.RTW_K_NAMES) if t.launches[i]),
            flush=True)
    world.close()
