#!/bin/bash
# Round-4 session 21: the first bounce's depth (max_depth) as a per-lane value too (build/rtw_cam.so) vs in-tree.
set -u
OUT=gpurun_out/s21
mkdir -p "$OUT"
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_cam.so || exit $?
CONFIG=c4 ROUNDS=1 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_cam.so || exit $?
CONFIG=c5 ROUNDS=1 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_cam.so || exit $?
