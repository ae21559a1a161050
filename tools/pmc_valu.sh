#!/bin/bash
# VALU issue counters of the bench's kernels (the VALU roofline of bench.py):
# one rocprofv3 --pmc pass, kernel-trace only, over `bench.py --steps 1 --warmup 0`
# (SQ counters <= 8, GRBM <= 2 per pass: MI355X_MICROARCH.md).
# Output: gpurun_out/pmc_valu/... and pmc_valu.json (tools/pmc_valu_summary.py);
# copy it to profiles/pmc_valu_<config>_<bvh>.json for bench.py.
set -u
OUT=${OUT:-gpurun_out/pmc_valu}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 1 --warmup 0"}
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
echo "== $CTRS"
timeout -k 10 600 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/valu" -o pmc -- python bench.py $ARGS > "$OUT/valu.log" 2>&1
rc=$?
echo "   rc=$rc"; tail -n 1 "$OUT/valu.log" | cut -c1-200
case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
python tools/pmc_valu_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
