#!/bin/bash
# Round-4 session 16: the RNG state in the 60-B layout's spare ray words (no rng stream) for scenes without
# ray time or media (build/rtw_rng.so): GPU suite on that library, then A/B vs in-tree on C4, Cornell, C2.
set -u
OUT=gpurun_out/s16
mkdir -p "$OUT"
RTW_LIB=build/rtw_rng.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread --deselect tests/test_abi.py::test_build_id_is_the_sources > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
CONFIG=c4 ROUNDS=2 STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_rng.so || exit $?
CONFIG=cornell ROUNDS=2 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_rng.so || exit $?
CONFIG=c2 ROUNDS=1 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_rng.so || exit $?
