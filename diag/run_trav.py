"""DIAGNOSTIC ONLY: drive diag/trav_bench.hip (traversal-only throughput).

Usage (GPU box): RTW_LIB=build/rtw_diag.so python diag/run_trav.py
"""
import ctypes as C
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

rtw = importlib.import_module("zig-raytracing-weekend_amd")
lib = rtw.lib()
lib.rtw_diag_trav.restype = C.c_int
lib.rtw_diag_trav.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.c_void_p,
                              C.POINTER(C.c_float)]

objs = rtw.worlds.generate_world(0, "book1")
cam = rtw.book1_camera().init()
out = torch.zeros(8, dtype=torch.int64, device="cuda")
for bvh in ("sah", "reference"):
    arr = rtw.flatten(objs, bvh_mode=rtw._abi.RTW_BVH_SAH if bvh == "sah" else rtw._abi.RTW_BVH_REFERENCE)
    w = rtw.World(arr)
    for mode, name in ((2, "lds/coherent"), (3, "global/coherent"), (6, "lds/coh+bounce"),
                       (7, "global/coh+bounce")):
        for blocks, rpl in ((8192, 8),):
            ms = C.c_float()
            for rep in range(3):
                out.zero_()
                rc = lib.rtw_diag_trav(w.handle, C.byref(cam.derived), mode, blocks, rpl, out.data_ptr(),
                                       C.byref(ms))
                assert rc == 0, rc
            torch.cuda.synchronize()
            rays = blocks * 256 * rpl
            nodes, leaves = int(out[0]), int(out[1])
            print(f"{bvh:9s} {name:16s} blocks={blocks:5d} rays={rays/1e6:6.2f}M ms={ms.value:8.3f} "
                  f"Grays/s={rays/ms.value/1e6:6.2f} nodes/ray={nodes/rays:6.1f} leaves/ray={leaves/rays:5.1f} "
                  f"Gnode/s={nodes/ms.value/1e6:7.1f}", flush=True)
    w.close()
