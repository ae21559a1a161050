#!/bin/bash
# PMC passes of ONE rank's shard at N ranks, for bench.py's roofline under torchrun (N > 1).
# A rank's launches cover ~1/N of the frame; pricing them with a whole-frame pass would read as a
# fraction > 1, so bench.py at N > 1 only uses profiles/pmc_{valu,traffic}_<config>_sah_n<N>_r<R>.json,
# taken here by rendering that shard alone on one GPU (bench.py --shard N,R: the same kernels, grid and
# rows as rank R of a torchrun job) and stamped with n_shards / rank by the summaries.
# Usage: tools/pmc_shard.sh <config> <N> <R>   -> gpurun_out/pmc_shard_<config>_n<N>_r<R>/
set -u
CFG=${1:-c2}; N=${2:-8}; R=${3:-0}
BASE=gpurun_out/pmc_shard_${CFG}_n${N}_r${R}
ARGS="--config $CFG --shard $N,$R --no-cpu-baseline --steps 1 --warmup 0"
OUT=$BASE/valu BENCH_ARGS="$ARGS" bash tools/pmc_valu.sh || exit $?
OUT=$BASE/traffic BENCH_ARGS="$ARGS" bash tools/pmc_traffic.sh || exit $?
cp "$BASE/valu/pmc_valu.json" "profiles/pmc_valu_${CFG}_sah_n${N}_r${R}.json"
cp "$BASE/traffic/pmc_traffic.json" "profiles/pmc_traffic_${CFG}_sah_n${N}_r${R}.json"
