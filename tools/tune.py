"""A/B timing of rtw_tuning settings on a config at reduced spp.
Usage: TUNE='[{"kernel": 1}, {"wf_iters": 12}, {"bvh": "ref"}]' python tools/tune.py [spp] [config]
Each setting: rtw_tuning fields (include/rtw_gpu.h) plus "bvh" ("sah"/"ref") and "order"."""
import ctypes as C
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

pkg = importlib.import_module("zig-raytracing-weekend_amd")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cfg_name = sys.argv[2] if len(sys.argv) > 2 else "c2"
settings = json.loads(os.environ.get("TUNE", '[{}, {"kernel": 1}, {"kernel": 2}]'))
cfg = pkg.configs.CONFIGS[cfg_name]
arr = pkg.flatten(cfg.objects())
cam = cfg.camera()
cam.samples_per_pixel = spp
cam.init()
acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
rounds = int(os.environ.get("TUNE_ROUNDS", "1"))  # round-robin repeats (box noise)
for st in [s for _ in range(rounds) for s in settings]:
    tun = dict(st)
    arr.bvh_mode = {"ref": 0, "sah": 1}[tun.pop("bvh", "sah")]
    arr.order_dir = tuple(tun.pop("order", (0.0, 0.0, 0.0)))
    world = pkg.World(arr, tuning=tun or None)
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # the render runs on `stream`: the zeroing must be done
    copts = pkg._abi.RtwRenderOpts(spp, 0, cnt.data_ptr())
    pkg._abi.check(pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0,
                                               acc.data_ptr(), C.c_void_p(stream.cuda_stream), C.byref(copts)), "count")
    c = cnt.cpu().tolist()
    st["nodes_per_ray"] = round((c[1] + c[2]) / max(1, c[0]), 2)
    st["inner_per_ray"] = round(c[1] / max(1, c[0]), 2)
    st["rays_per_sample"] = round(c[0] / (cam.size * 2), 3)
    opts = pkg._abi.RtwRenderOpts(spp, 0, None)
    best = 1e9
    for it in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rc = pkg.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0,
                                         acc.data_ptr(), C.c_void_p(stream.cuda_stream), C.byref(opts))
        pkg._abi.check(rc, "render")
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    print(json.dumps({"setting": st, "config": cfg_name, "spp": spp, "s": round(best, 4),
                      "Msamples_s": round(cam.size * spp / best / 1e6, 2)}), flush=True)
    world.close()
