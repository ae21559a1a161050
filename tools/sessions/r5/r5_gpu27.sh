#!/bin/bash
# Round 5: direction-bucketed queues on small batches (RTW_WF_SORT_MIN_CHUNKS 192 -> 0 / 96; library A/B:
# build/rtw_sort0.so, build/rtw_sort96.so = this commit with -DRTW_WF_SORT_MIN_CHUNKS=0u / 96u)
set -u
mkdir -p gpurun_out/r5
for spec in "c2 --shard 8,3" "c2 --tuning {\"wf_paths\":67108864}" "simple_light" "cornell" "cornell_smoke"; do
  set -- $spec; cfg=$1; shift; extra="$*"; tag=$(echo "$cfg$extra" | tr -c 'a-z0-9' '_' | cut -c1-40)
  OUT=gpurun_out/r5/ab_sortmin_$tag
  mkdir -p $OUT
  for r in 1 2; do
    for lib in "" build/rtw_sort0.so build/rtw_sort96.so; do
      t=$(basename "${lib:-default}" .so)
      RTW_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 3 --warmup 1 $extra > $OUT/${t}_$r.json 2> $OUT/err || { tail -5 $OUT/err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print('$tag', '$t', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
    done
  done
done
