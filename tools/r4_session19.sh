#!/bin/bash
# Round-4 session 19: C4 split trace -- same code, different contents of the ray records' spare words:
# build/rtw_zero.so (zeros) vs build/rtw_rnd.so (the RNG state's halves, random bits), vs in-tree.
set -u
OUT=gpurun_out/s19
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_zero.so build/rtw_rnd.so || exit $?
