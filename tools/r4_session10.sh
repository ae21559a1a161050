#!/bin/bash
# Round-4 session 10: -falign-loops=64 (build/rtw_a64.so) vs in-tree on C5, Cornell smoke, simple_light, C3.
set -u
OUT=gpurun_out/s10
mkdir -p "$OUT"
for c in c5 cornell_smoke simple_light; do CONFIG=$c ROUNDS=2 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?; done
CONFIG=c3 ROUNDS=1 STEPS=1 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?
