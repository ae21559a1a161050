#!/bin/bash
# Round 5: the full C2 batch without direction bucketing (sort_iters 0): does iteration 1 slow down per chunk as
# much as in a small batch?  per-launch traces
set -u
OUT=gpurun_out/r5/it1_probe2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "s3|" "s0|{\"sort_iters\":0}"; do
  n=${v%%|*}; tu=${v#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o kt -- python bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 1 ${tu:+--tuning "$tu"} > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
done
