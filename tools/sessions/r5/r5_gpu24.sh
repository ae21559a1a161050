#!/bin/bash
# Round 5: the tail in two launches (deal bit 64: 7 bounces per path, live paths requeued, then the rest) --
# bit identity, then A/Bs against deal 59 on C2 (N = 1 and rank 3 of 8), C4, Cornell, C5
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_objects.py tests/test_gpu_multi.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "knobs_invariant or deal or objects or shard or c3_geometry or fused_step" > gpurun_out/r5/gpu24_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu24_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab_tail2_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=3 STEPS=5 bash tools/ab_knob.sh '' '{"deal": 123}' || exit 1
OUT=gpurun_out/r5/ab_tail2_c2 CONFIG=c2 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"deal": 123}' || exit 1
OUT=gpurun_out/r5/ab_tail2_c4 CONFIG=c4 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"deal": 123}' || exit 1
OUT=gpurun_out/r5/ab_tail2_cornell CONFIG=cornell ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"deal": 123}' || exit 1
OUT=gpurun_out/r5/ab_tail2_c5 CONFIG=c5 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"deal": 123}' || exit 1
