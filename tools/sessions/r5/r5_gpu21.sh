#!/bin/bash
# Round 5: dynamic claims in the split kernels (C4) and the wavefront-iteration count under deal 59 (1|2|8|16|32)
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_objects.py tests/test_gpu_multi.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "knobs_invariant or deal or objects or shard or c3_geometry or fused_step or compact_nodes" > gpurun_out/r5/gpu21_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu21_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab_deal7_c4 CONFIG=c4 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"deal": 51}' '{"deal": 59}' || exit 1
OUT=gpurun_out/r5/ab_iters3_c2 CONFIG=c2 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"deal": 59}' '{"deal": 59, "wf_iters": 5}' '{"deal": 59, "wf_iters": 6}' '{"deal": 59, "wf_iters": 9}' || exit 1
OUT=gpurun_out/r5/ab_iters3_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '{"deal": 59}' '{"deal": 59, "wf_iters": 6}' '{"deal": 59, "wf_iters": 9}' || exit 1
OUT=gpurun_out/r5/ab_iters3_cornell CONFIG=cornell ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"deal": 59}' '{"deal": 59, "wf_iters": 6}' || exit 1
