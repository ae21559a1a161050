#!/bin/bash
# Round 5: where the per-rank fixed cost at N ranks goes -- every rank's shard of C2 rendered
# alone on this GPU by bench.py --shard N,R (the torchrun rank's exact launches), per-kernel HIP-event times.
# usage: bash tools/r5_shard_breakdown.sh [config] [N] [tuning-json]
set -u
CFG=${1:-c2}; N=${2:-8}; TU=${3:-}
OUT=gpurun_out/r5/shard_${CFG}_n${N}${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 ${TU:+--tuning "$TU"} > $OUT/n1.json 2> $OUT/err || { tail $OUT/err; exit 1; }
for r in $(seq 0 $((N-1))); do
  timeout -k 10 300 python bench.py --config $CFG --shard $N,$r --no-cpu-baseline --steps 3 --warmup 1 ${TU:+--tuning "$TU"} \
    > $OUT/r$r.json 2> $OUT/err || { tail $OUT/err; exit 1; }
done
python - "$OUT" "$N" <<'PY'
import json, sys
d, n = sys.argv[1], int(sys.argv[2])
one = json.load(open(f"{d}/n1.json"))
print("N=1", one["ms_per_step"], one["roofline"]["kernel_ms_per_step"], one["roofline"]["launches"])
worst = 0
for r in range(n):
    x = json.load(open(f"{d}/r{r}.json"))
    worst = max(worst, x["ms_per_step"])
    print(f"rank {r}", x["ms_per_step"], x["roofline"]["kernel_ms_per_step"], "rows", x["config"]["shard"]["rows"])
print("predicted speedup", round(one["ms_per_step"] / worst, 3), "ideal per rank", round(one["ms_per_step"] / n, 3), "worst", worst)
PY
