#!/usr/bin/env python3
"""Where the compact walk's wave steps go (diagnostic build: make -C zig-raytracing-weekend_amd/csrc diag).

Renders a config at reduced spp through build/rtw_diag.so and prints, over every compact walk of the
render (the fused step's bounce walks, tiles over the list cap, the tail):
  lane util of the walk   = lane steps / (64 * wave steps)
  leaf share of steps     = wave steps where some lane tests a sphere
  exact share of steps    = wave steps where some lane runs the exact-root path
  exact lanes that hit    = exact-path entries that moved `closest` (the rest: estimate undecided, no hit)
Usage: RTW_LIB=build/rtw_diag.so python tools/diag_walk.py [config] [spp] [tuning-json]
"""
import ctypes as C
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("RTW_LIB", os.path.join(REPO, "build", "rtw_diag.so"))


def main():
    import torch
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    tun = json.loads(sys.argv[3]) if len(sys.argv) > 3 else None
    pkg = importlib.import_module("zig-raytracing-weekend_amd")
    L = pkg.lib()
    fn = L.rtw_debug_walk_counters
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    cfg = pkg.configs.CONFIGS[cfg_name]
    arr = pkg.flatten(cfg.objects())
    world = pkg.World(arr, tuning=tun)
    cam = cfg.camera()
    cam.samples_per_pixel = spp
    cam.init()
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    out = (C.c_uint64 * 16)()
    fn(out, 1)
    rc = L.rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0, acc.data_ptr(), None, None)
    pkg._abi.check(rc, "rtw_render_device")
    torch.cuda.synchronize()
    fn(out, 1)
    ws, wl, we, ls, ll, le, leh, walks = list(out)[:8]
    lw, lc, lwalk, lex = list(out)[8:12]
    res = {"config": cfg_name, "spp": spp, "walks": walks, "wave_steps": ws, "lane_steps": ls,
           "lane_util_walk": ls / max(1, 64 * ws), "steps_per_walk": ls / max(1, walks),
           "leaf_share_of_wave_steps": wl / max(1, ws), "exact_share_of_wave_steps": we / max(1, ws),
           "leaf_share_of_lane_steps": ll / max(1, ls), "exact_lanes_per_walk": le / max(1, walks),
           "exact_lanes_that_hit": leh / max(1, le), "lanes_per_exact_step": le / max(1, we),
           "lanes_per_leaf_step": ll / max(1, wl),
           "list_waves": lw, "list_waves_over_cap": lwalk, "list_candidates_per_wave": lc / max(1, lw),
           "list_exact_candidates_per_wave": lex / max(1, lw)}
    print(json.dumps(res))
    world.close()


if __name__ == "__main__":
    main()
