"""DIAGNOSTIC ONLY: per-wave start / stage-done / end times of the C2 fused step and tail.  The stamps are not in
the product sources (they would change its build id): apply diag/wave_stamps.patch to a checkout, then
`make -C zig-raytracing-weekend_amd/csrc variant NAME=wstamps DEFS=-DRTW_WAVE_STAMPS` -> build/rtw_wstamps.so.

Usage (GPU box): RTW_LIB=build/rtw_wstamps.so python diag/run_wave_stamps.py [n_shards rank] [out.json]
Renders C2 (or one rank's shard) twice, reads the stamps of the second render and prints, per launch: the spread
of wave starts (ramp), the LDS stage time, and the end-time distribution (drain) relative to the launch."""
import ctypes as C
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

rtw = importlib.import_module("zig-raytracing-weekend_amd")
lib = rtw.lib()
lib.rtw_diag_wave_stamps.restype = C.c_int
lib.rtw_diag_wave_stamps.argtypes = [C.c_void_p, C.c_size_t]
n_shards = int(sys.argv[1]) if len(sys.argv) > 2 else 1
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
out_path = sys.argv[3] if len(sys.argv) > 3 else ""
cfg = rtw.configs.CONFIGS["c2"]
world = rtw.World(rtw.flatten(cfg.objects()))
cam = cfg.camera().init()
spp = cam.samples_per_pixel
WAVES = 8192
buf = np.zeros(16 * WAVES * 4, dtype=np.uint64)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
if n_shards > 1:
    sh = rtw.distributed.ShardedRender(world, cam, rank, n_shards, 8 | rtw._abi.RTW_ROWS_BALANCED)
    render = lambda: sh.render(0, spp, stream=stream)  # noqa: E731
else:
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")

    def render():
        rtw._abi.check(lib.rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 0,
                                             acc.data_ptr(), C.c_void_p(stream.cuda_stream), None), "render")
for k in range(2):
    render()
    torch.cuda.synchronize()
    assert lib.rtw_diag_wave_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(16, WAVES, 4).astype(np.float64) * 10.0 / 1e3  # 100 MHz ticks -> microseconds
res = {"n_shards": n_shards, "rank": rank, "build_id": lib.rtw_build_id().decode(), "launches": {}}
for slot in range(16):
    s = st[slot]
    live = s[:, 0] > 0
    if not live.any():
        continue
    s = s[live]
    t0 = s[:, 0].min()
    start, staged, end = s[:, 0] - t0, s[:, 1] - t0, s[:, 2] - t0
    d = {"waves": int(live.sum()), "start_max": float(start.max()), "start_p50": float(np.median(start)),
         "stage_done_p50": float(np.median(staged[staged > -1e8])) if (s[:, 1] > 0).any() else None,
         "end_min": float(end.min()), "end_p10": float(np.percentile(end, 10)), "end_p50": float(np.median(end)),
         "end_p90": float(np.percentile(end, 90)), "end_p99": float(np.percentile(end, 99)), "end_max": float(end.max())}
    res["launches"]["tail" if slot == 15 else f"it{slot}"] = d
    print(slot, json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items()}))
if out_path:
    json.dump(res, open(out_path, "w"), indent=1)
