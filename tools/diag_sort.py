#!/usr/bin/env python3
"""Would sorting the bounce rays help the walk?  (a global sort of the survivor queue.)

Diagnostic build only (make -C zig-raytracing-weekend_amd/csrc diag -> build/rtw_diag.so).  One render of
a config at reduced spp records, for every compact walk of wavefront iteration `it`, the walk's step count
and its ray (rtw_debug_walk_records: per path slot).  The waves of that iteration take their rays 64
consecutive slots at a time, so grouping the records by slot // 64 reproduces the actual waves, and

    walk lane utilisation = sum of steps / (64 * sum over waves of the longest walk)

is what the hardware paid.  The same is computed for the rays regrouped in 64s after sorting the whole
queue (a global sort) or each 4096-slot window (a windowed sort) by keys a sort could use: octant,
direction bins, origin cells, both; a random order (no coherence) and the walk length itself (the bound no
key can beat) frame them.  Prints one JSON line.
Usage: RTW_LIB=build/rtw_diag.so python tools/diag_sort.py [config] [spp] [iteration]
"""
import ctypes as C
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("RTW_LIB", os.path.join(REPO, "build", "rtw_diag.so"))


def util(steps, groups):
    """steps: float tensor in lane order; groups: group id per lane (64-lane waves)."""
    import torch
    ng = int(groups.max().item()) + 1
    mx = torch.zeros(ng, device=steps.device).scatter_reduce_(0, groups, steps, reduce="amax")
    return float(steps.sum() / (64.0 * mx.sum()))


def main():
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    it = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    pkg = importlib.import_module("zig-raytracing-weekend_amd")
    L = pkg.lib()
    L.rtw_debug_walk_records.restype = C.c_int
    L.rtw_debug_walk_records.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    cfg = pkg.configs.CONFIGS[name]
    world = pkg.World(pkg.flatten(cfg.objects()))
    cam = cfg.camera()
    cam.samples_per_pixel = spp
    cam.init()
    paths = ((cam.derived.image_width + 7) // 8 * 8) * ((cam.derived.image_height + 7) // 8 * 8) * spp
    cap = 2 * paths + (1 << 20)
    rec = torch.zeros((cap, 8), dtype=torch.int32, device="cuda")
    pkg._abi.check(L.rtw_debug_walk_records(rec.data_ptr(), cap, it), "rtw_debug_walk_records")
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    rc = L.rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0, acc.data_ptr(), None, None)
    pkg._abi.check(rc, "rtw_render_device")
    torch.cuda.synchronize()
    pkg._abi.check(L.rtw_debug_walk_records(None, 0, 0xFFFFFFFF), "rtw_debug_walk_records")
    valid = rec[:, 7] != 0
    slot = torch.nonzero(valid).squeeze(1)
    r = rec[slot]
    steps = (r[:, 0] & 0xFFFF).float()
    d = r[:, 1:4].view(torch.float32)
    o = r[:, 4:7].view(torch.float32)
    n = steps.numel()
    out = {"config": name, "spp": spp, "iteration": it, "walks": n, "mean_steps": float(steps.mean())}
    out["actual_waves"] = util(steps, slot // 64)

    seq = torch.arange(n, device="cuda")
    dn = d / d.norm(dim=1, keepdim=True)
    oct_ = (d[:, 0] < 0).long() | ((d[:, 1] < 0).long() << 1) | ((d[:, 2] < 0).long() << 2)
    dbin = ((dn + 1) * 4).clamp(0, 7.999).long()                       # 8 bins per axis of the unit direction
    dkey = dbin[:, 0] * 64 + dbin[:, 1] * 8 + dbin[:, 2]
    elev = ((dn[:, 1] + 1) * 8).clamp(0, 15.999).long()               # 16 elevation bins
    cell = torch.floor(o).long()                                      # 1-unit origin cells
    pid = (r[:, 7] - 1).long()
    tile = (pid // 64) // spp                                         # the camera tile (tile-major path ids)
    ckey = ((cell[:, 0] + 2048) * 4096 + (cell[:, 1] + 2048)) * 4096 + (cell[:, 2] + 2048)
    keys = {
        "random": torch.randperm(n, device="cuda"),
        "octant": oct_,
        "elevation16": elev,
        "direction512": dkey,
        "origin_cell": ckey,
        "origin_cell+octant": ckey * 8 + oct_,
        "origin_cell+direction512": ckey * 512 + dkey,
        "walk_length (bound)": steps.long(),
        "tile": tile,
        "tile+octant": tile * 8 + oct_,
        "tile+direction512": tile * 512 + dkey,
        "tile+direction64": tile * 64 + (dbin[:, 0] // 2) * 16 + (dbin[:, 1] // 2) * 4 + dbin[:, 2] // 2,
        "tile4x4+direction512": ((tile // 150) // 4 * 38 + (tile % 150) // 4) * 512 + dkey,
        "tile+direction16": tile * 16 + oct_ * 2 + (dbin[:, 1] >= 4).long(),
        "tile+direction32": tile * 32 + oct_ * 4 + (dbin[:, 1] // 2) % 4,
    }
    if os.environ.get("DIAG_SORT_KEYS"):
        keep = set(os.environ["DIAG_SORT_KEYS"].split(","))
        keys = {k: v for k, v in keys.items() if k in keep}
    glob_res, win_res = {}, {}
    for kname, k in keys.items():
        k = torch.unique(k, return_inverse=True)[1]  # dense keys 0..m-1 (no overflow in the window key)
        order = torch.argsort(k, stable=True)        # stable: ties keep the queue order
        glob_res[kname] = util(steps[order], seq // 64)
        # windowed: sort within consecutive 4096-slot windows of the queue (the round-1 experiment's form)
        wk = (slot // 4096) * (int(k.max().item()) + 1) + k
        order = torch.argsort(wk, stable=True)
        win_res[kname] = util(steps[order], seq // 64)
    out["global_sort"] = glob_res
    out["window4096_sort"] = win_res
    print(json.dumps(out))
    world.close()


if __name__ == "__main__":
    main()
