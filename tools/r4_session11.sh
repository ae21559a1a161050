#!/bin/bash
# Round-4 session 11: GPU suite on the in-tree build (loop alignment + the defocus disk's cooperative
# rejection loop), then A/B against build/rtw_a64.so (loop alignment only) on C2 and C4.
set -u
OUT=gpurun_out/s11
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { cat "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?
CONFIG=c4 ROUNDS=1 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?
