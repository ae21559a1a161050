#!/bin/bash
# Round 5: dynamic tail input (deal 1) -- bit-identity (every knob under deal 1), then the N=8 breakdown.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shard or multi or c3_geometry or knobs_invariant or four_copy or objects or smoke" > gpurun_out/r5/gpu8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu8_tests.txt; [ $rc = 0 ] || exit $rc
TAG=tail_deal1 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1}' || exit 1
for cfg in c4 cornell; do
  OUT=gpurun_out/r5/ab_deal_$cfg CONFIG=$cfg ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"deal": 1}' || exit 1
done
