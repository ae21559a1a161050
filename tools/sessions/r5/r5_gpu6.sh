#!/bin/bash
# Round 5: guided dealing (single chunks at the end of iteration 0) + batched reduce loads; N=8 breakdown
# under wavefront iteration counts 9 / 12 / 16 (how much of the tail's excess at 8 ranks is its longest paths).
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shard or multi or c3_geometry or knobs_invariant or full_size or reduce" > gpurun_out/r5/gpu6_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu6_tests.txt; [ $rc = 0 ] || exit $rc
TAG=g_deal1 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1}' || exit 1
TAG=g_deal1_it12 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1, "wf_iters": 12}' || exit 1
TAG=g_deal1_it16 bash tools/r5_shard_breakdown.sh c2 8 '{"deal": 1, "wf_iters": 16}' || exit 1
