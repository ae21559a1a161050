#!/bin/bash
# Round 5: deal bits 16 (fused iterations >= 1 claimed per stripe group) and 32 (16 x waves singles at the end of
# iteration 0) -- bit identity, then same-box A/Bs at N = 1 and on rank 3 of 8 (C2), C4, Cornell
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_objects.py tests/test_gpu_multi.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "knobs_invariant or deal or objects or shard or c3_geometry or fused_step" > gpurun_out/r5/gpu19_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu19_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab_deal5_c2 CONFIG=c2 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"deal": 35}' '{"deal": 19}' '{"deal": 51}' || exit 1
OUT=gpurun_out/r5/ab_deal5_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=3 STEPS=5 bash tools/ab_knob.sh '' '{"deal": 35}' '{"deal": 19}' '{"deal": 51}' || exit 1
OUT=gpurun_out/r5/ab_deal5_c4 CONFIG=c4 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"deal": 35}' || exit 1
OUT=gpurun_out/r5/ab_deal5_cornell CONFIG=cornell ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"deal": 35}' '{"deal": 19}' '{"deal": 51}' || exit 1
