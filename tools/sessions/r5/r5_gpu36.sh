#!/bin/bash
# Round 5: the scalar-unit bucketed push (build/rtw_pushs.so = this commit with -DRTW_PUSH_SCALAR) -- same images
# (C3-geometry test: bucketing on, against the oracle; full C2 frame against the in-tree library), then A/Bs
set -u
OUT=gpurun_out/r5/ab_pushs; mkdir -p $OUT
RTW_LIB=build/rtw_pushs.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 \
  --timeout-method thread -k "c3_geometry or knobs_invariant or fused_step or four_copy" > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt; [ $rc = 0 ] || exit $rc
for lib in "" build/rtw_pushs.so; do
  t=$(basename "${lib:-default}" .so)
  RTW_LIB=$lib timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 0 --dump-image $OUT/img_$t.npy > /dev/null 2> $OUT/err || { tail $OUT/err; exit 1; }
done
python -c "
import numpy as np, hashlib
a=np.load('$OUT/img_default.npy'); b=np.load('$OUT/img_rtw_pushs.npy')
print('frames identical:', np.array_equal(a, b), a.shape, hashlib.sha256(a.tobytes()).hexdigest()[:16], hashlib.sha256(b.tobytes()).hexdigest()[:16])
assert np.array_equal(a, b)" || exit 1
rm -f $OUT/img_*.npy
for cfg in c2 c4 c5 c3; do
  st=3; [ $cfg = c4 ] && st=2; [ $cfg = c5 ] && st=2; [ $cfg = c3 ] && st=1
  OUT2=$OUT/$cfg; mkdir -p $OUT2
  for r in 1 2; do
    for lib in "" build/rtw_pushs.so; do
      t=$(basename "${lib:-default}" .so)
      RTW_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps $st --warmup 1 > $OUT2/${t}_$r.json 2> $OUT/err || { tail $OUT/err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT2/${t}_$r.json'));print('$cfg', '$t', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
    done
  done
done
