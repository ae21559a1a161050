#!/bin/bash
# Round-4 final measurement of the build with the packed state in the split kernels and the RNG state in the
# 60-B records (per-lane iteration depth): GPU suite + smoke + build-stamped PMC + bench lines
# (tools/r4_final2.sh), then same-box A/Bs against the previous final build (build/rtw_base.so).
set -u
bash tools/r4_final2.sh || exit $?
OUT=gpurun_out/r4/ab
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
CONFIG=cornell ROUNDS=2 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
CONFIG=c2 ROUNDS=1 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_base.so || exit $?
