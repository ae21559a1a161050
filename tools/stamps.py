"""Diagnostic: per-phase wave-cycle split of the persistent kernel (RTW_STAMPS build).
Run with RTW_LIB=build/rtw_stamps.so.  Shares only, never timings."""
import ctypes as C
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

pkg = importlib.import_module("zig-raytracing-weekend_amd")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = pkg.configs.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c2"]
arr = pkg.flatten(cfg.objects())
cam = cfg.camera()
cam.samples_per_pixel = spp
cam.init()
world = pkg.World(arr)
acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
opts = pkg._abi.RtwRenderOpts(spp, 0, cnt.data_ptr())
pkg._abi.check(pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0,
                                           acc.data_ptr(), None, C.byref(opts)), "render")
torch.cuda.synchronize()
c = cnt.cpu().tolist()
tot = sum(c[8:12])
names = ["assign", "gen", "trav", "shade"]
print({n: round(c[8 + i] / tot, 4) for i, n in enumerate(names)})
print("trav steps per pass", round(c[12] / max(1, c[13]), 2), "passes", c[13], "rays", c[0],
      "lane-steps/wave-step", round((c[1] + c[2]) / max(1, c[12]), 2))
