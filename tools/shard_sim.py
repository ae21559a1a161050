"""Predict strong-scaling of the row-interleaved multi-GPU render on ONE GPU.

For N in (1, 2, 4, 8) renders every rank's shard (rtw_render_rows_device, the
call bench.py makes per rank) back to back on this GPU and reports the slowest
rank's render time: the N-GPU step time minus the RCCL gather (C2: 15.4 MB,
~1-2 ms over xGMI).  Usage: [RTW_SHARD_TUNING=json] python tools/shard_sim.py [config] [spp] [rows_per_block] [ranks, e.g. 1,8]
"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

pkg = importlib.import_module("zig-raytracing-weekend_amd")
cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
spp_override = int(sys.argv[2]) if len(sys.argv) > 2 else 0
# default: bench.py's split (8-row blocks, balanced residual rows, RTW_ROWS_BALANCED); 0x80000008 = the same explicitly
rpb = int(sys.argv[3], 0) if len(sys.argv) > 3 else 8 | pkg._abi.RTW_ROWS_BALANCED
ns = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 4, 8]
cfg = pkg.configs.CONFIGS[cfg_name]
# RTW_SHARD_TUNING='{"wf_iters": 16}': the rtw_tuning fields to override (every setting renders the same image)
world = pkg.World(pkg.flatten(cfg.objects()), tuning=json.loads(os.environ.get("RTW_SHARD_TUNING", "{}")))
cam = cfg.camera()
if spp_override:
    cam.samples_per_pixel = spp_override
cam.init()
spp = cam.samples_per_pixel
W, H = cam.derived.image_width, cam.derived.image_height
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
base = None
for n in ns:
    times = []
    for r in range(n if n > 1 else 1):
        sh = pkg.distributed.ShardedRender(world, cam, r, n, rpb)
        sh.render(0, spp, stream=stream)           # warm-up (allocates wavefront state)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            sh.render(0, spp, stream=stream)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        times.append(best)
        del sh
    slow = max(times)
    if base is None:
        base = slow
    print(json.dumps({"config": cfg_name, "n": n, "rows_per_block": rpb & 0xFFFF,
                      "balanced": bool(rpb & pkg._abi.RTW_ROWS_BALANCED), "build_id": pkg.lib().rtw_build_id().decode(), "rank_ms": [round(t * 1e3, 2) for t in times],
                      "max_ms": round(slow * 1e3, 2), "pred_speedup": round(base / slow, 3),
                      "pred_Msamples_s": round(W * H * spp / slow / 1e6, 1)}), flush=True)
world.close()
