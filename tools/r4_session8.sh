#!/bin/bash
# Round-4 session 8: code placement. Loop headers aligned to 64 B (-falign-loops=64: build/rtw_a64.so), and the
# split kernels on the packed path state with and without it (build/rtw_pk.so, build/rtw_pk_a64.so), vs in-tree.
set -u
OUT=gpurun_out/s8
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=1 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_pk.so build/rtw_pk_a64.so build/rtw_a64.so || exit $?
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?
CONFIG=cornell ROUNDS=1 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?
