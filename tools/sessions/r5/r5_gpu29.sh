#!/bin/bash
# Round 5: only iteration 0 bucketed (sort_iters 1), on every batch size (build/rtw_sort0.so: threshold 0) --
# against the default (sort_iters 3 on batches of >= 192 chunks per wave) on every config
set -u
OUT=gpurun_out/r5/ab_sort1; mkdir -p $OUT
for spec in "c2" "c2 --shard 8,3" "simple_light" "cornell" "cornell_smoke" "c5" "c4"; do
  set -- $spec; cfg=$1; shift; extra="$*"; tag=$(echo "$cfg$extra" | tr -c 'a-z0-9' '_' | cut -c1-30)
  st=3; [ $cfg = c4 ] && st=2; [ $cfg = c5 ] && st=2; [ "$extra" != "" ] && st=5
  for r in 1 2; do
    for v in "default|" "default|{\"sort_iters\":1}" "sort0|{\"sort_iters\":1}"; do
      lib=${v%%|*}; tu=${v#*|}; L=""; [ $lib = sort0 ] && L=build/rtw_sort0.so
      t=$(echo "${tag}_${lib}_$tu" | tr -c 'a-z0-9_' '_')
      RTW_LIB=$L timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps $st --warmup 1 $extra ${tu:+--tuning "$tu"} > $OUT/${t}_$r.json 2> $OUT/err || { tail -5 $OUT/err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print('$t', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
    done
  done
done
