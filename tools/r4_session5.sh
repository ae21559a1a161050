#!/bin/bash
# Round-4 session 5: GPU suite on the per-render layout flag, then same-box A/Bs: C2 in-tree vs the
# leaf-postponing walks (build/rtw_lp{4,8}.so), C4 split path 60-B state (default) vs packed (fuse bit 8).
set -u
OUT=gpurun_out/s5
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_lp4.so build/rtw_lp8.so || exit $?
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_knob.sh '' '{"fuse": 11}' || exit $?
