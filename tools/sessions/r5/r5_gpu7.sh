#!/bin/bash
# Round 5: balanced rows with alternating round order -- bit-identity, then the N=8 rank breakdown.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shard or multi or c3_geometry" > gpurun_out/r5/gpu7_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu7_tests.txt; [ $rc = 0 ] || exit $rc
TAG=alt_deal1 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1}' || exit 1
TAG=alt_deal1 bash tools/r5_shard_breakdown.sh c2 4 '{"deal": 1}' || exit 1
TAG=alt_deal1 bash tools/r5_shard_breakdown.sh c2 2 '{"deal": 1}' || exit 1
mkdir -p gpurun_out/r5/walk
RTW_LIB=build/rtw_trav.so timeout -k 10 300 python diag/run_walk_ceiling.py c2 gpurun_out/r5/walk/ceiling_c2.json > gpurun_out/r5/walk/c2.log 2>&1 || { tail gpurun_out/r5/walk/c2.log; exit 1; }
cat gpurun_out/r5/walk/c2.log
