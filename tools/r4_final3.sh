#!/bin/bash
# Round-4 final measurement (split translation units): GPU suite + smoke, tools/final_r4.sh, then same-box
# A/Bs of the in-tree build against build/rtw_a64.so (whole library with 64-B loop alignment).
set -u
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r4/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/r4/gpu_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.txt 2>&1 || { cat gpurun_out/r4/smoke.txt; exit 1; }
tail -1 gpurun_out/r4/smoke.txt
bash tools/final_r4.sh || exit $?
OUT=gpurun_out/r4/ab
for c in simple_light c2; do CONFIG=$c ROUNDS=2 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_a64.so || exit $?; done
