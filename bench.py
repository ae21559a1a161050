#!/usr/bin/env python3
"""Benchmark: Msamples/s of the path-tracing hot path on BASELINE config 2
(Book-1 random spheres, 1200x800, 500 spp, depth 50).

A "step" = one complete render of the configuration: every pixel x every
sample, through the C ABI (rtw_render_rows_device) into an HBM-resident float4
accumulator, plus (N > 1) the RCCL gather of the row-interleaved shards to
rank 0 and their reassembly.  Scene build / BVH / upload happen once, before
timing.  N GPUs split the same image (strong scaling): rank r renders row
blocks b with b % N == r.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
       (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N_SIMD = 256 * 4               # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9               # max engine clock (MI355X_MICROARCH.md)
# VALU issue ceiling, measured on the box (diag/valu_peak.hip -> profiles/r4_valu_peak/): independent
# v_fma_f32 / v_add_f32 chains at 8 waves/SIMD issue one wave64 instruction per SIMD every 2.09 / 2.06
# clocks (74.7 / 75.8 T lane-op/s at the 2.37-2.38 GHz the chip holds), as MI355X_MICROARCH.md:54,473
# state; v_pk_fma_f32 takes 4 clocks (the same lane-FMA rate).  Peak = 32 lanes per SIMD per clock.
VALU_CYCLES_PER_INST = 2.0
VALU_PEAK_TLOPS = round(N_SIMD * 64 / VALU_CYCLES_PER_INST * CLOCK_HZ / 1e12, 3)   # 78.643 T lane-op/s
VALU_PEAK_SRC = "profiles/r4_valu_peak/summary.txt"
NODE_BYTES = 32                # one BVH node / leaf record (rtw_layout.h)
ROWS_PER_BLOCK = 8   # row blocks interleaved over ranks: C2 at 8 GPUs 6.97x predicted (16: 6.87x; tools/shard_sim.py)
# the rows left over after whole rounds of blocks split evenly (RTW_ROWS_BALANCED): C2 at 8 ranks renders 100 rows per
# rank instead of 104 on four ranks and 96 on the others (profiles/r5_shard/)
ROWS_BALANCED = True


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--single-process", action="store_true",
                    help="drive the N GPUs from this one process through the C ABI (rtw_multi: shard renders + one "
                         "grouped RCCL send/recv); without it, --gpus N > 1 needs torchrun (one process per GPU)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2",
                    choices=["c1", "c2", "c3", "c4", "c5", "cornell", "cornell_smoke", "simple_light"])
    ap.add_argument("--spp", type=int, default=0, help="override spp (0 = config's)")
    ap.add_argument("--bvh", default="sah", choices=["sah", "reference"])
    ap.add_argument("--tuning", default="", help='rtw_tuning fields as JSON, e.g. {"wf_iters": 12} (A/B only)')
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline duration")
    ap.add_argument("--cpu-threads", type=int, default=8, help="reference uses 8 render threads (main.zig:41)")
    ap.add_argument("--host-backend", action="store_true",
                    help="render every rank's shard on a host context (RTW_DEVICE_CPU, rtw_render_rows) and gather "
                         "over gloo: the same torchrun flow (shards, gather, reassembly, timing, JSON line) with no "
                         "GPU, for the CPU tests; never a headline number")
    ap.add_argument("--host-threads", type=int, default=2, help="--host-backend: render threads per rank")
    ap.add_argument("--dump-image", default="", help="rank 0 saves the reassembled float4 frame (.npy)")
    ap.add_argument("--shard", default="",
                    help="N,R: render only rank R's shard of an N-way split on this one GPU, no gather (the PMC "
                         "passes of one rank at N, tools/pmc_shard.sh; never a headline number)")
    ap.add_argument("--profiles-dir", default=os.path.join(REPO, "profiles"),
                    help="where the committed PMC passes are read from (tests point it elsewhere)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    single = args.single_process
    if world_size > 1 and (single or world_size != args.gpus):
        raise SystemExit("torchrun: --gpus must equal the number of ranks and excludes --single-process")
    if world_size == 1 and args.gpus > 1 and not single:
        raise SystemExit("--gpus N > 1: launch one process per GPU with torchrun (the driver's scaling run), or "
                         "pass --single-process for the one-process rtw_multi path")
    n_shards = args.gpus if single else world_size
    shard_rank = rank
    emulated = bool(args.shard)
    if emulated:  # one rank's shard of an N-way split, rendered alone on this GPU
        if world_size > 1 or single or args.gpus > 1 or args.dump_image:
            raise SystemExit("--shard N,R runs one process on one GPU (no torchrun, --single-process or --dump-image)")
        n_shards, shard_rank = (int(v) for v in args.shard.split(","))
        if not (n_shards >= 1 and 0 <= shard_rank < n_shards):
            raise SystemExit("--shard N,R needs 0 <= R < N")
    host = args.host_backend
    if host and single:
        raise SystemExit("--host-backend is the torchrun (one process per rank) flow")
    if not host:
        torch.cuda.set_device(local_rank)
    distributed = world_size > 1
    if distributed:  # backend "nccl" is RCCL on ROCm; gloo carries the host-backend rehearsal
        if host:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def sync():
        if not host:
            torch.cuda.synchronize()

    pkg = importlib.import_module("zig-raytracing-weekend_amd")
    L = pkg.lib()
    # (an A/B build of an ABI before 6, RTW_LIB=..., has no build id: its rooflines are not derived anyway)
    build_id = L.rtw_build_id().decode() if hasattr(L, "rtw_build_id") else "pre-abi6"
    cfg = pkg.configs.CONFIGS[args.config]
    objs = cfg.objects()
    bvh_mode = {"sah": pkg._abi.RTW_BVH_SAH, "reference": pkg._abi.RTW_BVH_REFERENCE}[args.bvh]
    arr = pkg.flatten(objs, bvh_mode=bvh_mode)
    t0 = time.time()
    tun = json.loads(args.tuning) if args.tuning else None
    if host:
        tun = dict(tun or {}, cpu_threads=args.host_threads)
    world = pkg.World(arr, device=pkg._abi.RTW_DEVICE_CPU if host else local_rank, tuning=tun)
    # single-process multi-GPU: one context per device + the RCCL communicators of rtw_multi
    worlds = [world] + [pkg.World(arr, device=k, tuning=tun) for k in range(1, n_shards)] if single else [world]
    rpb_arg = ROWS_PER_BLOCK | (pkg._abi.RTW_ROWS_BALANCED if ROWS_BALANCED else 0)
    multi = pkg.distributed.MultiDeviceRender(worlds, rpb_arg) if single else None
    # the exchange's participants as the collective layer reports them: rtw_multi's RCCL communicator
    # (ncclCommCount), or torch.distributed's process group (backend "nccl" = RCCL on ROCm)
    if single:
        rccl = {"mode": "rtw_multi", "rccl_ranks": multi.info()[1], "backend": "rccl (ncclCommInitAll)"}
    elif distributed:
        rccl = {"mode": "torchrun", "rccl_ranks": dist.get_world_size(), "backend": str(dist.get_backend())}
    else:
        rccl = {"mode": "single_gpu", "rccl_ranks": None, "backend": None}
    build_s = time.time() - t0
    # the reference topology (bvh.zig) defines the algorithmic bytes
    world_ref = None if host else pkg.World(pkg.flatten(objs, bvh_mode=pkg._abi.RTW_BVH_REFERENCE), device=local_rank)
    cam = cfg.camera()
    if args.spp:
        cam.samples_per_pixel = args.spp
    cam.init()
    W, H, spp = cam.derived.image_width, cam.derived.image_height, cam.samples_per_pixel
    stats = world.stats()

    stream = None if host else torch.cuda.Stream()  # explicit stream: the kernels and the timing events share it
    if not host:
        torch.cuda.set_stream(stream)
    # the shard this process renders (single-process mode: device 0's, for the counted and timing passes)
    shard = pkg.distributed.ShardedRender(world, cam, shard_rank, n_shards, rpb_arg,
                                          device=torch.device("cpu") if host else None)
    my_rows = shard.rows
    assert my_rows == L.rtw_shard_rows(H, rpb_arg, n_shards, shard_rank)
    frame = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda") if single else None

    def render_step(counters=None, w=None, timing=None):
        if w is not None:
            saved, shard.world = shard.world, w
        shard.render(0, spp, seed=0, stream=stream, counters=counters, timing=timing)
        if w is not None:
            shard.world = saved

    def gather_step():
        if not single and not emulated:
            shard.gather()

    def frame_step():
        # one whole frame: every shard rendered + gathered (single-process: rtw_render_multi_device)
        if single:
            multi.render_device(cam, 0, spp, frame.data_ptr(), seed=0, stream=stream, fresh=True, sync=False)
        else:
            render_step()

    # ---- algorithmic bytes of one step: counted pass on the reference topology (the device
    # walk of a reference-topology tree visits exactly the nodes bvh.zig's recursion visits)
    def counted(w):
        keys = ("nodes", "leaves", "rays", "samples", "nan", "tail_rays")
        if host:  # host contexts keep no device counters
            return dict.fromkeys(keys, 0)
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        render_step(cnt.data_ptr(), w)
        torch.cuda.synchronize()
        c = cnt.cpu().numpy()
        return {k: int(c[getattr(pkg._abi, "RTW_STAT_" + k.upper())]) for k in keys}
    cref = counted(world_ref)
    cdev = counted(world)
    if world_ref is not None:
        world_ref.close()
    nodes, leaves, rays, samples = cref["nodes"], cref["leaves"], cref["rays"], cref["samples"]
    nan_count = cdev["nan"]
    pixels = my_rows * W
    alg_bytes = NODE_BYTES * (nodes + leaves) + 32 * pixels

    for _ in range(args.warmup):
        frame_step()
        gather_step()
    sync()

    # per-kernel HIP events, recorded by the library on the render stream around every launch
    timings = [pkg._abi.RtwKernelTiming() for _ in range(args.steps)]
    ev = ([] if host else
          [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)])
    host_ms = []
    if distributed:
        dist.barrier()
    sync()
    t_start = time.perf_counter()
    for k in range(args.steps):
        if host:
            t0k = time.perf_counter()
            render_step()
            host_ms.append((time.perf_counter() - t0k) * 1e3)
        else:
            ev[k][0].record(stream)
            if single:
                frame_step()
            else:
                render_step(timing=timings[k])
            ev[k][1].record(stream)
        gather_step()
    sync()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kernel_ms = host_ms if host else [a.elapsed_time(b) for a, b in ev]
    if single:  # per-kernel HIP events of device 0's shard, rendered alone after the timed region
        for k in range(args.steps):
            render_step(timing=timings[k])
        torch.cuda.synchronize()
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if host else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.dump_image and rank == 0:  # the reassembled frame (world size 1: this rank's tile is the frame)
        if not distributed:
            shard.gather()
        np.save(args.dump_image, shard.image.cpu().numpy())

    if single:
        multi.close()
        for w in worlds[1:]:
            w.close()
    total_samples = (my_rows if emulated else H) * W * spp * args.steps
    value = total_samples / elapsed / 1e6
    render_s = sum(kernel_ms) / len(kernel_ms) / 1e3          # whole render call (all kernels) per step
    kms = {n: sum(t.ms[i] for t in timings) for i, n in enumerate(pkg._abi.RTW_K_NAMES)}
    kcalls = {n: sum(t.launches[i] for t in timings) for i, n in enumerate(pkg._abi.RTW_K_NAMES)}
    dom = max(kms, key=lambda n: kms[n])                        # dominant kernel (device time)
    # algorithmic bytes (reference topology) of the rays each kernel kind traces
    b_ray = NODE_BYTES * (nodes + leaves) / max(1, rays)
    # (SURVEY §8d prices traversal; a shading-dominated config -- Perlin/image textures, c5 -- has no
    # algorithmic-byte model here: achieved/frac are null rather than a misleading 0)
    dom_bytes_step = {"trace": b_ray * (rays - cref["tail_rays"]), "tail": b_ray * cref["tail_rays"],
                      "mega": alg_bytes}.get(dom)
    dom_launch_s = kms[dom] / max(1, kcalls[dom]) / 1e3
    dom_bytes_launch = dom_bytes_step * args.steps / max(1, kcalls[dom]) if dom_bytes_step is not None else None
    achieved = dom_bytes_launch / dom_launch_s / 1e9 if (dom_bytes_launch is not None and dom_launch_s > 0) else None
    path_achieved = alg_bytes / render_s / 1e9
    # fused path (compact LDS stage): one gen+trace+shade kernel per iteration, timed as "trace"
    fused = kcalls["trace"] > 0 and kcalls["shade"] == 0
    knames = {"trace": "wf_step_clds" if fused else "wf_trace", "tail": "wf_tail", "mega": "render_persistent_v1"}
    # (the PMC passes are per shard: at N > 1 only a pass of this rank's shard at this N -- bench.py --shard N,R
    # on one GPU, tools/pmc_shard.sh -- prices this rank's launches; anything else leaves the fractions null)
    # (host backend: the lookup runs -- the CPU tests check it -- but there are no device launch times, so
    # every fraction below stays null)
    traffic, traffic_src = pmc_traffic(
        args, {"trace": "wf_step" if fused else "wf_trace", "tail": "wf_tail", "mega": "render_"}.get(dom, dom),
        build_id, n_shards, shard_rank, single)

    # ---- roofline of the dominant kernel: VALU issue.  The kernel is VALU-bound
    # (C2: VALU busy 0.85 of the quad-cycles, HBM 0.18 of peak), so `frac` = useful lane-instructions
    # per second / the non-packed VALU issue peak; lane-instructions per launch come from the
    # committed SQ pass of this bench (tools/pmc_valu.sh -> profiles/pmc_valu_<config>_<bvh>.json),
    # the launch time is this run's HIP events.  HBM traffic (PMC) and the SURVEY §8d algorithmic
    # bytes are reported beside it; the latter is a diagnostic, not a fraction of any peak.
    dom_kind = {"trace": "wf_step" if fused else "wf_trace", "tail": "wf_tail", "mega": "render_"}.get(dom, dom)
    valu, valu_src = pmc_valu(args, dom_kind, build_id, n_shards, shard_rank, single)
    if host:
        dom_launch_s = 0.0
    lane_ops = valu.get("lane_ops") if valu else None
    achieved_valu = lane_ops / dom_launch_s / 1e12 if (lane_ops and dom_launch_s > 0) else None
    # fraction of the SIMD cycles spent issuing VALU at the measured 2-clock wave64 rate
    issue = (valu["insts_valu"] * VALU_CYCLES_PER_INST / (N_SIMD * dom_launch_s * CLOCK_HZ)
             if (valu and dom_launch_s > 0) else None)
    hbm_achieved = traffic / dom_launch_s / 1e9 if (traffic and dom_launch_s > 0) else None
    roofline = {
        "bound": "valu",
        "achieved": round(achieved_valu, 3) if achieved_valu is not None else None,
        "peak": VALU_PEAK_TLOPS,
        "unit": "Tlane-op/s",
        "frac": round(achieved_valu / VALU_PEAK_TLOPS, 4) if achieved_valu is not None else None,
        "traffic": traffic,
        # the dominant kernel's instantiations as the committed PMC pass of this config recorded them (round 6:
        # iteration 0 and the later iterations of a step are two instantiations; the launch time and the PMC
        # figures are averages over both)
        "kernel": (" + ".join(valu["kernels"]) if valu and valu.get("kernels") else knames.get(dom, dom)),
        "kernels": (list(valu["kernels"]) if valu and valu.get("kernels") else [knames.get(dom, dom)]),
        "fused_step": fused,
        "avg_launch_ms": round(dom_launch_s * 1e3, 4),
        "launches_per_step": kcalls[dom] / args.steps,
        "valu": {"source": valu_src, "kind": dom_kind, "lane_ops_per_launch": lane_ops,
                 "lane_util": round(valu["lane_util"], 4) if valu else None,
                 "issue_busy": round(issue, 4) if issue is not None else None,
                 "peak_def": "256 CU x 4 SIMD x 32 lanes x 2.4 GHz: one wave64 VALU instruction per SIMD every 2 "
                             "clocks, measured at 8 waves/SIMD (v_fma_f32 2.09, v_add_f32 2.06 clocks); = the "
                             "157.3 TFLOP/s datasheet figure / 2 flops per FMA",
                 "peak_source": VALU_PEAK_SRC,
                 "build_id": build_id,
                 "frac_of_fp32_fma_peak": round(achieved_valu * 2 / 157.3, 4) if achieved_valu else None},
        "hbm": {"achieved": round(hbm_achieved, 2) if hbm_achieved is not None else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(hbm_achieved / HBM_PEAK_GBS, 4) if hbm_achieved is not None else None,
                "traffic_per_launch": traffic, "source": traffic_src, "kind": dom_kind, "build_id": build_id},
        "kernel_ms_per_step": {n: round(v / args.steps, 3) for n, v in kms.items() if kcalls[n]},
        "launches": {n: v // args.steps for n, v in kcalls.items() if v},
        "algorithmic": {"note": "SURVEY 8d bytes of the reference-topology walk (53 nodes/ray x 32 B) per second; "
                                "the tree is LDS-resident and the SAH walk visits 23 nodes/ray, so this is not a "
                                "fraction of HBM peak",
                        "bytes_per_s_dominant": round(achieved, 2) if achieved is not None else None,
                        "alg_bytes_per_launch": round(dom_bytes_launch) if dom_bytes_launch is not None else None,
                        "path_bytes_per_s": round(path_achieved, 2), "render_ms": round(render_s * 1e3, 3),
                        "alg_bytes_per_step": alg_bytes,
                        "alg_bytes_per_sample": round(alg_bytes / max(1, samples), 2),
                        "alg_bytes_per_ray": round(b_ray, 2)},
        "rays_per_sample": round(rays / max(1, samples), 4),
        "tail_ray_frac": round(cref["tail_rays"] / max(1, rays), 5),
        "nodes_per_ray_reference": round((nodes + leaves) / max(1, rays), 3),
        "nodes_per_ray_device": round((cdev["nodes"] + cdev["leaves"]) / max(1, cdev["rays"]), 3),
        "bvh": args.bvh,
    }
    # ---- the work-normalised walk roofline: the render's device node visits (inner boxes +
    # sphere tests of the SAH walk, the counted pass) per second against the walk ceiling -- the same compact
    # LDS walk alone on the config's camera (+ bounce) rays, measured on this build (diag/trav_bench.hip,
    # diag/run_walk_ceiling.py -> profiles/walk_ceiling_<config>.json).  Redundant lanes (the cooperative
    # rejection loop's idle-lane candidates, hoisted spheres every lane tests) do not count here: a visit is
    # one lane's step of its own walk.
    dev_steps = cdev["nodes"] + cdev["leaves"]
    walk_achieved = dev_steps / render_s if (render_s > 0 and not host) else None
    ceiling, ceil_src = walk_ceiling(args, build_id)
    roofline["walk"] = {
        "unit": "node-steps/s", "achieved": walk_achieved, "ceiling": ceiling,
        "frac": round(walk_achieved / ceiling, 4) if (walk_achieved and ceiling) else None,
        "device_steps_per_render": dev_steps, "render_ms": round(render_s * 1e3, 3), "source": ceil_src,
        "note": "device walk steps (inner boxes + sphere tests, one lane's own walk each) of a whole render per "
                "second of render, over the compact LDS walk's rate alone on the config's rays (the ceiling)"}
    # A VALU or HBM fraction above 1 is physically impossible: pmc_pass only prices this build's own shard, so it
    # means a wrong PMC pass, peak or launch time -- a measurement bug.  The raw value stays in the line, the
    # section carries "error", and the run exits non-zero after printing it (tests/test_bench_contract.py).  The
    # walk ceiling is a measured rate, not a hardware peak: a walk fraction above 1 is reported as it is.
    frac_errors = []
    for name, sec in (("valu", roofline), ("hbm", roofline["hbm"])):
        if sec["frac"] is not None and sec["frac"] > 1.0:
            sec["error"] = (f"{name} frac {sec['frac']} > 1 from {sec.get('source') or roofline['valu']['source']}: "
                            "a measurement bug")
            frac_errors.append(sec["error"])

    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(pkg, arr, cam, args)

    if rank == 0:
        line = {
            "metric": ("Msamples/s (pixel·spp) on 1200×800 Book-1 random-spheres @500spp; 1→8 GPU"
                       if args.config == "c2" else f"Msamples/s (pixel·spp) on {cfg.description}"),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": n_shards,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded %s scene (%d world objects), counter-based RNG seed 0" % (args.config, len(objs)),
            "config": {"workload": cfg.description, "config_id": args.config, "width": W, "height": H,
                       "spp": spp, "max_depth": cam.max_depth, "objects": len(objs), "bvh_nodes": stats["n_nodes"],
                       "bvh_depth": stats["depth"], "parallelism": f"row-interleaved tiles x{n_shards}"
                       + ((" + gloo gather (host backend)" if host else " + RCCL gather") if distributed else "")
                       + (" (one process, rtw_multi: grouped RCCL send/recv)" if single else ""),
                       "rows_per_block": ROWS_PER_BLOCK, "row_split": "balanced" if ROWS_BALANCED else "blocks",
                       "exchange": rccl,
                       "shard": {"n_shards": n_shards, "rank": shard_rank, "rows": my_rows,
                                 "emulated": emulated},
                       "timed_scope": ("host contexts (rtw_render_rows) into host tiles, gathered over gloo: the "
                                       "CPU rehearsal of the torchrun flow" if host else
                                       "device API (rtw_render_rows_device / rtw_render_multi_device) into an "
                                       "HBM-resident float4 accumulator; no host copy inside the timed region")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "nan_samples": nan_count,
            "scene_build_s": round(build_s, 4),
            "build_id": build_id,
        }
        print(json.dumps(line), flush=True)
    world.close()
    if distributed:
        dist.destroy_process_group()
    if frac_errors:
        print("bench.py: " + "; ".join(frac_errors), file=sys.stderr, flush=True)
        sys.exit(3)


def pmc_build_id(data):
    """The rtw_build_id() of the library a committed PMC pass was taken on (tools/pmc_*_summary.py)."""
    b = data.get("_build") if isinstance(data, dict) else None
    return b.get("build_id") if isinstance(b, dict) else None


def pmc_pass(args, kind, build_id, n_shards=1, rank=0, single=False):
    """The committed PMC pass of `kind` ("valu" | "traffic") that prices THIS process's launches, or
    (None, reason).  A pass counts one launch of the shard it was taken on: N = 1 the whole frame
    (profiles/pmc_<kind>_<config>_<bvh>.json), N > 1 rank R's rows of an N-way split, rendered alone on
    one GPU (bench.py --shard N,R: profiles/pmc_<kind>_<config>_<bvh>_n<N>_r<R>.json, stamped with
    n_shards / rank).  Never another shard's pass: at N = 8 the whole-frame counts over a rank's ~1/6.5-length
    launch would read as a fraction > 1.  Nor a pass of another library build, an A/B run (--spp, --tuning,
    RTW_LIB) or the single-process multi path (other kernels)."""
    if args.spp or args.tuning or single or os.environ.get("RTW_LIB"):
        return None, None
    suffix = f"_n{n_shards}_r{rank}" if n_shards > 1 else ""
    f = os.path.join(args.profiles_dir, f"pmc_{kind}_{args.config}_{args.bvh}{suffix}.json")
    rel = os.path.relpath(f, REPO)
    if not os.path.exists(f):
        return None, (f"{rel}: no pass of this rank's shard at N = {n_shards} (fractions null)" if n_shards > 1
                      else None)
    data = json.load(open(f))
    if pmc_build_id(data) != build_id:
        return None, f"{rel}: build {pmc_build_id(data)} != loaded {build_id} (stale, unused)"
    b = data.get("_build") or {}
    if (int(b.get("n_shards") or 1), int(b.get("rank") or 0)) != (n_shards, rank):
        return None, f"{rel}: pass of shard {b.get('rank')}/{b.get('n_shards')}, not {rank}/{n_shards} (unused)"
    return data, rel


def pmc_traffic(args, kernel_prefix, build_id, n_shards=1, rank=0, single=False):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (tools/pmc_traffic.sh -> profiles/pmc_traffic_<config>_<bvh>[_n<N>_r<R>].json; FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md § HBM).  PMC counters cannot be read inside the timed run (pmc_pass)."""
    data, src = pmc_pass(args, "traffic", build_id, n_shards, rank, single)
    if data is None:
        return None, src
    for name, e in data.items():
        if name.startswith(kernel_prefix) and isinstance(e, dict):
            return round(e["traffic_bytes"]), src
    return None, None


def pmc_valu(args, kind, build_id, n_shards=1, rank=0, single=False):
    """VALU counters per launch of the dominant kernel kind from the committed SQ pass
    (tools/pmc_valu.sh -> profiles/pmc_valu_<config>_<bvh>[_n<N>_r<R>].json).  Returns (entry, path)."""
    data, src = pmc_pass(args, "valu", build_id, n_shards, rank, single)
    if data is None:
        return None, src
    for name, e in data.items():
        if name.startswith(kind) and isinstance(e, dict) and e.get("lane_ops"):
            return e, src
    return None, None


def walk_ceiling(args, build_id):
    """The walk ceiling of this config measured on this build (diag/run_walk_ceiling.py ->
    profiles/walk_ceiling_<config>.json), or (None, reason).  The ceiling belongs to one build: a file of
    another build is unused, and A/B runs (--spp, --tuning, --bvh other than sah, RTW_LIB builds) get none.
    Shards at N > 1 do get it: the walk rate is node-steps per second of render, which a shard's shorter
    render does not change, unlike the per-launch PMC counts of pmc_pass."""
    if args.spp or args.tuning or args.bvh != "sah" or os.environ.get("RTW_LIB"):
        return None, None
    f = os.path.join(args.profiles_dir, f"walk_ceiling_{args.config}.json")
    if not os.path.exists(f):
        return None, None
    d = json.load(open(f))
    rel = os.path.relpath(f, REPO)
    if d.get("build_id") != build_id:
        return None, f"{rel}: build {d.get('build_id')} != loaded {build_id} (stale, unused)"
    return d["ceiling"], rel


def cpu_quota_cores():
    """CPUs this process may use: the cgroup v2 quota (cpu.max) when set, else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(pkg, arr, cam, args):
    """The C oracle (faithful restatement, oracle/) on the host: samples-outer
    loop over contiguous chunks with the reference's 8 render threads, on every
    8th image row (a bounded, row-representative sample of the same scene and
    camera), with spp scaled to ~args.cpu_seconds."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O

    ow = O.World.from_arrays(arr)
    d = cam.derived
    ocam = O.camera(aspect_ratio=cam.aspect_ratio, image_width=d.image_width, image_height=d.image_height,
                    samples_per_pixel=d.samples_per_pixel, max_depth=d.max_depth, background=tuple(d.background),
                    background_mode=d.background_mode, vfov=cam.vfov, lookfrom=cam.lookfrom, lookat=cam.lookat,
                    vup=cam.vup, defocus_angle=cam.defocus_angle, focus_dist=cam.focus_dist,
                    pixel_offset=d.pixel_offset)
    W, H = d.image_width, d.image_height
    rows = np.arange(0, H, 8)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    quota = cpu_quota_cores()
    legs = {}
    for name, th in (("threads_8", args.cpu_threads), ("threads_quota", quota), ("threads_all", os.cpu_count() or 1)):
        if any(v["threads"] == th for v in legs.values()):
            legs[name] = dict(next(v for v in legs.values() if v["threads"] == th))
            continue
        t = time.perf_counter()
        ow.render_pixels(ocam, 0, pix, 0, 1, threads=th)
        t1 = time.perf_counter() - t
        spp = int(max(1, min(d.samples_per_pixel, args.cpu_seconds / max(t1, 1e-3))))
        t = time.perf_counter()
        ow.render_pixels(ocam, 0, pix, 0, spp, threads=th)
        dt = time.perf_counter() - t
        legs[name] = {"threads": th, "value": round(len(pix) * spp / dt / 1e6, 4), "spp": spp, "seconds": round(dt, 2)}
    best = max(legs.values(), key=lambda v: v["value"])
    return {"value": best["value"], "unit": "Msamples/s", "cores": best["threads"], "kind": "port",
            "sample": f"every 8th row of {W}x{H} ({len(pix)} px), contiguous size/threads chunks "
                      f"(main.zig:318-324), spp scaled to ~{args.cpu_seconds:.0f} s per leg; legs: 8 threads "
                      f"(main.zig:41), the cgroup CPU quota ({quota} CPUs), and os.cpu_count() "
                      f"({os.cpu_count()}) threads; value = the fastest leg",
            "legs": legs, "cores_all": os.cpu_count(), "cpu_quota_cores": quota}


if __name__ == "__main__":
    main()
