#!/bin/bash
# Round-4 session 13: octant copies of the compact-node LDS stage staggered across the banks (in-tree) vs the
# final build (build/rtw_final.so): GPU suite first, then C2 x2 and C3.
set -u
OUT=gpurun_out/s13
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_final.so || exit $?
CONFIG=c3 ROUNDS=1 STEPS=1 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_final.so || exit $?
