import ctypes as C, importlib, os, sys
import numpy as np
sys.path.insert(0, '.')
import torch
rtw = importlib.import_module("zig-raytracing-weekend_amd")
cfg = rtw.configs.CONFIGS["c4"]
arr = rtw.flatten(cfg.objects())
cam = cfg.camera(); cam.samples_per_pixel = 2; cam.init()
acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
for o in ("1", "8", "1", "8"):
    os.environ["RTW_ORDERS"] = o
    w = rtw.World(arr)
    for rep in range(2):
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        opts = rtw._abi.RtwRenderOpts(2, 0, cnt.data_ptr())
        rtw._abi.check(rtw.lib().rtw_render_device(w.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0, acc.data_ptr(), None, C.byref(opts)), "r")
        torch.cuda.synchronize()
        print(o, rep, cnt.cpu().numpy().tolist(), flush=True)
    w.close()
