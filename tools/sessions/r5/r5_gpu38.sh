#!/bin/bash
# Round 5: C4's tail (wf_tail_w5, 41 % of the step) at 4 / 5 / 6 waves per SIMD (build/rtw_tw4.so, rtw_tw6.so = this
# commit with -DRTW_TAIL_WAVES=4 / 6; default 5)
set -u
OUT=gpurun_out/r5/ab_tailwaves_c4; mkdir -p $OUT
for r in 1 2; do
  for lib in "" build/rtw_tw6.so build/rtw_tw4.so; do
    t=$(basename "${lib:-default}" .so)
    RTW_LIB=$lib timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/${t}_$r.json 2> $OUT/err || { tail $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${t}_$r.json'));print('c4', '$t', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
