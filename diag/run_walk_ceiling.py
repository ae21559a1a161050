"""DIAGNOSTIC ONLY: the walk ceiling of the compact LDS walk (diag/trav_bench.hip, built by `make -C
zig-raytracing-weekend_amd/csrc trav` into build/rtw_trav.so) on a config's scene and camera rays.

Usage (GPU box): RTW_LIB=build/rtw_trav.so python diag/run_walk_ceiling.py [config] [out.json] [tuning-json]
Prints one JSON line per ray mode and writes {"build_id", "config", "modes": {...}, "ceiling": ...} to out.json:
the ceiling is the best node-steps/s (inner boxes + sphere tests) of the walk alone, which bench.py's
roofline.walk compares with the product's device node visits per second on the same build."""
import ctypes as C
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

rtw = importlib.import_module("zig-raytracing-weekend_amd")
lib = rtw.lib()
lib.rtw_diag_walk_ceiling.restype = C.c_int
lib.rtw_diag_walk_ceiling.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                      C.POINTER(C.c_float), C.POINTER(C.c_uint32)]
cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
out_path = sys.argv[2] if len(sys.argv) > 2 else ""
tuning = json.loads(sys.argv[3]) if len(sys.argv) > 3 else None
cfg = rtw.configs.CONFIGS[cfg_name]
w = rtw.World(rtw.flatten(cfg.objects()), tuning=tuning)
cam = cfg.camera().init()
out = torch.zeros(8, dtype=torch.int64, device="cuda")
res = {"build_id": lib.rtw_build_id().decode(), "config": cfg_name, "tuning": tuning, "modes": {}}
for bounce, name in ((0, "camera"), (1, "camera+bounce")):
    best = None
    for rep in range(4):
        out.zero_()
        ms, grid = C.c_float(), C.c_uint32()
        rc = lib.rtw_diag_walk_ceiling(w.handle, C.byref(cam.derived), 64, bounce, out.data_ptr(), C.byref(ms),
                                       C.byref(grid))
        assert rc == 0, rc
        torch.cuda.synchronize()
        nodes, leaves, walks = (int(v) for v in out[:3].tolist())
        if rep == 0:
            continue  # warm-up
        rate = (nodes + leaves) / (ms.value / 1e3)
        if best is None or rate > best["steps_per_s"]:
            best = {"steps_per_s": rate, "nodes": nodes, "leaves": leaves, "walks": walks, "ms": ms.value,
                    "grid": grid.value, "steps_per_walk": (nodes + leaves) / max(1, walks)}
    res["modes"][name] = best
    print(json.dumps({"mode": name, **best}), flush=True)
res["ceiling"] = max(m["steps_per_s"] for m in res["modes"].values())
res["note"] = ("node-steps/s (inner boxes + sphere tests) of the compact LDS walk alone, one 1024-thread block "
               "per CU, on the config's camera rays of 8x8 tiles (+ one diffuse bounce); the best mode")
if out_path:
    json.dump(res, open(out_path, "w"), indent=1)
w.close()
