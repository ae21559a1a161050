#!/bin/bash
# Round 5: balanced shard rows (RTW_ROWS_BALANCED) + dynamic deal -- bit-identity, then the N=8 rank breakdown.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shard or multi or c3_geometry or knobs_invariant or boundary" > gpurun_out/r5/gpu5_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu5_tests.txt; [ $rc = 0 ] || exit $rc
TAG=bal_deal1 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1}' || exit 1
TAG=bal_deal0 bash tools/r5_shard_breakdown.sh c2 8 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_native_harness.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r5/gpu5_native.txt 2>&1
tail -3 gpurun_out/r5/gpu5_native.txt
