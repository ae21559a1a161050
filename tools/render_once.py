#!/usr/bin/env python3
"""One render of a config through the device API (for profilers: PC sampling, counters).
Usage: python tools/render_once.py [config] [spp] [tuning-json]"""
import ctypes as C
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    tun = json.loads(sys.argv[3]) if len(sys.argv) > 3 else None
    pkg = importlib.import_module("zig-raytracing-weekend_amd")
    cfg = pkg.configs.CONFIGS[name]
    world = pkg.World(pkg.flatten(cfg.objects()), tuning=tun)
    cam = cfg.camera()
    cam.samples_per_pixel = spp
    cam.init()
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    rc = pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0, acc.data_ptr(),
                                     None, None)
    pkg._abi.check(rc, "rtw_render_device")
    torch.cuda.synchronize()
    print(f"rendered {name} {cam.size} px x {spp} spp")
    world.close()


if __name__ == "__main__":
    main()
