#!/bin/bash
# Strong-scaling prediction of the final build (every rank's shard rendered alone on this GPU): C3 and C2.
set -u
mkdir -p gpurun_out/shard
timeout -k 10 300 python tools/shard_sim.py c3 0 8 1,2,4,8 > gpurun_out/shard/c3.jsonl 2> gpurun_out/shard/c3.err || { tail -5 gpurun_out/shard/c3.err; exit 1; }
timeout -k 10 300 python tools/shard_sim.py c2 0 8 1,2,4,8 > gpurun_out/shard/c2.jsonl 2> gpurun_out/shard/c2.err || { tail -5 gpurun_out/shard/c2.err; exit 1; }
cat gpurun_out/shard/c3.jsonl gpurun_out/shard/c2.jsonl
