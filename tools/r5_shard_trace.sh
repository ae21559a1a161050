#!/bin/bash
# kernel trace of C2 at N=1 and of rank R of N (bench.py --shard): per-launch durations by iteration
set -u
N=${1:-8}; R=${2:-3}; TU=${3:-}
OUT=gpurun_out/r5/shard_trace${TAG:+_$TAG}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/n1 -o kt -- python bench.py --config c2 --no-cpu-baseline --steps 2 --warmup 1 ${TU:+--tuning "$TU"} > $OUT/n1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r$R -o kt -- python bench.py --config c2 --shard $N,$R --no-cpu-baseline --steps 2 --warmup 1 ${TU:+--tuning "$TU"} > $OUT/r$R.log 2>&1 || exit $?
