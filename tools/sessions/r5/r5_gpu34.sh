#!/bin/bash
# Round 5: C3 (3840x2160 x 1024 spp, BASELINE's 8-GPU config) shard predictions on the final build
set -u
mkdir -p gpurun_out/r5f
timeout -k 10 900 python tools/shard_sim.py c3 > gpurun_out/r5f/c3_shard_sim.jsonl 2> gpurun_out/r5f/c3_shard_sim.err || { tail gpurun_out/r5f/c3_shard_sim.err; exit 1; }
cat gpurun_out/r5f/c3_shard_sim.jsonl
