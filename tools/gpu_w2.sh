#!/bin/bash
# A/B of rtw_tuning settings on one config (diagnostic): parity subset, then one bench per tuning.
#   CFG=c4 TUNINGS='{"wide_walk": 1}|{"wide_walk": 0}' bash tools/gpu_w2.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c4}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "${TESTK:-knobs_invariant or compact_nodes or stress or fast_reject}" > gpurun_out/pt_w2.log 2>&1
  rc=$?; tail -3 gpurun_out/pt_w2.log; [ $rc -le 1 ] || exit $rc
fi
IFS='|' read -ra TU <<< "${TUNINGS:-{\"wide_walk\": 1\}|{\"wide_walk\": 0\}}"
k=0
for t in "${TU[@]}"; do
  timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --steps ${STEPS:-2} --warmup 1 --tuning "$t" > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_$k.json'));r=d['roofline'];print(sys.argv[1], d['value'], r['kernel_ms_per_step'])" "$t"
  k=$((k+1))
done
