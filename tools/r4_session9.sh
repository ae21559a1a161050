#!/bin/bash
# Round-4 session 9: C4 with the cooperative rejection loop in the split shade and the L1/L2 tail too
# (build/rtw_coopall.so, built with -falign-loops=64) vs in-tree and build/rtw_a64.so.
set -u
OUT=gpurun_out/s9
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so build/rtw_coopall.so || exit $?
