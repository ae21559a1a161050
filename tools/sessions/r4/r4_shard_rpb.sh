#!/bin/bash
# C2 at 1 / 8 ranks with 4-row blocks (200 blocks: 25 per rank at 8 ranks) vs 8-row blocks.
set -u
mkdir -p gpurun_out/shard
for rpb in 4 8; do
  timeout -k 10 200 python tools/shard_sim.py c2 0 $rpb 1,2,4,8 > gpurun_out/shard/c2_rpb$rpb.jsonl 2> gpurun_out/shard/c2_rpb$rpb.err || { tail -5 gpurun_out/shard/c2_rpb$rpb.err; exit 1; }
  echo "rpb $rpb"; cat gpurun_out/shard/c2_rpb$rpb.jsonl
done
