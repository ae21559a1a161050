#!/bin/bash
# Round-4 session 3: C2 A/B of the leaf-postponing walk variants (build/rtw_lp{2,4}.so) against the in-tree
# library, then C4 per-iteration kernel times of the in-tree library and build/rtw_head.so.
set -u
OUT=gpurun_out/s3
mkdir -p "$OUT"
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_lp2.so build/rtw_lp4.so || exit $?
for lib in "" build/rtw_head.so; do
  tag=$(basename "${lib:-default}" .so)
  RTW_LIB=$lib OUT=$OUT/it_$tag CONFIG=c4 SPP=64 bash tools/iter_ab.sh '' || exit $?
done
