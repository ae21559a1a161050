#!/bin/bash
# Round-4 session 12: C4 with the split kernels on the packed state and full 16-B ray loads (build/rtw_p1.so)
set -u
OUT=gpurun_out/s12
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_p1.so || exit $?
