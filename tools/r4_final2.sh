#!/bin/bash
# Round-4 final measurement on the final build: GPU suite + smoke, then tools/final_r4.sh (build-stamped PMC
# passes of all 7 configs copied into profiles/ on the box, bench lines, C2 rocprof summary, stall passes).
set -u
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r4/gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/r4/gpu_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.txt 2>&1 || { cat gpurun_out/r4/smoke.txt; exit 1; }
tail -1 gpurun_out/r4/smoke.txt
bash tools/final_r4.sh
