#!/bin/bash
# Round-4 session 18: C4 split trace -- in-tree vs liveness from the direction bits on the unchanged 60-B
# layout (build/rtw_live.so) vs the RNG-in-ray-words layout (build/rtw_rng.so): code or data?
set -u
OUT=gpurun_out/s18
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_live.so build/rtw_rng.so || exit $?
