#!/bin/bash
# C2 at 1 and 8 ranks (shard_sim) with 9 / 16 / 24 / 50 wavefront iterations before the tail.
set -u
mkdir -p gpurun_out/shard
for it in 9 16 24 50; do
  RTW_SHARD_TUNING="{\"wf_iters\": $it}" timeout -k 10 200 python tools/shard_sim.py c2 0 8 1,8 > gpurun_out/shard/c2_it$it.jsonl 2> gpurun_out/shard/c2_it$it.err || { tail -5 gpurun_out/shard/c2_it$it.err; exit 1; }
  echo "wf_iters $it"; cat gpurun_out/shard/c2_it$it.jsonl
done
