#!/bin/bash
# Round 5: auto wf_iters (4 / 9 on image textures) -- whole GPU suite, bench lines, C2 8-rank shard breakdown
set -u
bash tools/sessions/r5/r5_gpu9.sh || exit 1
TAG=iters_auto bash tools/r5_shard_breakdown.sh c2 8
# four-wide records: same hits, then C4 A/B against the in-tree (two-wide) library
RTW_LIB=build/rtw_wide4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "compact_nodes_are_exact or knobs_invariant or far or l1" > gpurun_out/r5/wide4_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/wide4_tests.txt; [ $rc = 0 ] || exit $rc
RTW_LIB=build/rtw_wide4s.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "compact_nodes_are_exact" > gpurun_out/r5/wide4s_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/wide4s_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab_wide4_c4 CONFIG=c4 ROUNDS=2 STEPS=2 bash tools/ab_c2.sh "" build/rtw_wide4.so build/rtw_wide4s.so
