#!/bin/bash
# Round 5: per-launch traces to locate iteration 1's excess on a shard -- the full frame in 8 batches (wf_paths 2^26)
# vs rank 3 of 8, with and without the camera-ray tile lists
set -u
OUT=gpurun_out/r5/it1_probe; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o kt -- python bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 1 "$@" > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
}
run n1
run n1_b8 --tuning '{"wf_paths": 67108864}'
run r3 --shard 8,3
run r3_notl --shard 8,3 --tuning '{"tile_lists": 0}'
run r3_s0 --shard 8,3 --tuning '{"sort_iters": 0}'
