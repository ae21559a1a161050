#!/bin/bash
# Round 5: dynamic dealing of iteration 0 (tuning.deal) -- bit-identity, then N=1 and N=8 rank A/B.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "knobs_invariant or shard or c3_geometry" > gpurun_out/r5/gpu4_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu4_tests.txt; [ $rc = 0 ] || exit $rc
TAG=deal0 bash tools/r5_shard_breakdown.sh c2 8 || exit 1
TAG=deal1 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1}' || exit 1
