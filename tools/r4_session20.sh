#!/bin/bash
# Round-4 session 20: the split trace with the iteration depth made a per-lane value (asm VGPR barrier):
# build/rtw_rngv.so (RNG state in the 60-B records' spare words) and build/rtw_pkv.so (packed split state),
# C4 A/B vs in-tree, then Cornell for rngv.
set -u
OUT=gpurun_out/s20
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_rngv.so build/rtw_pkv.so || exit $?
