#!/bin/bash
# Round-4 session 15: the 60-B layout's path id folded into thr.w (no separate pid stream) in-tree vs the
# final build (build/rtw_base.so): GPU suite, then C4 x2, Cornell, C2.
set -u
OUT=gpurun_out/s15
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
CONFIG=cornell ROUNDS=2 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
CONFIG=c2 ROUNDS=1 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
