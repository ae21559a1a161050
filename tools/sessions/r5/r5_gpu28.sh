#!/bin/bash
# Round 5: bucketing on a shard with fewer buckets / fewer sorted iterations (build/rtw_sort0.so: threshold 0),
# plus per-launch traces of default vs sort0 on rank 3 of 8
set -u
OUT=gpurun_out/r5/ab_sort0_r3; mkdir -p $OUT
for r in 1 2; do
  for spec in "default|" "sort0|" "sort0|{\"sort_bits\":2}" "sort0|{\"sort_bits\":3}" "sort0|{\"sort_iters\":1}" "sort0|{\"sort_iters\":1,\"sort_bits\":2}"; do
    lib=${spec%%|*}; tu=${spec#*|}; L=""; [ $lib = sort0 ] && L=build/rtw_sort0.so
    t=$(echo "${lib}_$tu" | tr -c 'a-z0-9_' '_')
    RTW_LIB=$L timeout -k 10 300 python bench.py --config c2 --shard 8,3 --no-cpu-baseline --steps 5 --warmup 1 ${tu:+--tuning "$tu"} > $OUT/${t}_$r.json 2> $OUT/err || { tail -5 $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print('$t', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in default sort0; do
  L=""; [ $lib = sort0 ] && L=build/rtw_sort0.so
  RTW_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$lib -o kt -- python bench.py --config c2 --shard 8,3 --no-cpu-baseline --steps 1 --warmup 1 > $OUT/trace_$lib.log 2>&1 || { tail $OUT/trace_$lib.log; exit 1; }
done
