#!/bin/bash
# The gfx950 VALU issue ceiling (diag/valu_peak.hip): one plain run (HIP-event rates), then one
# rocprofv3 --pmc pass (SQ + GRBM counters per dispatch, kernel-trace only) over the same binary.
# Output: $OUT/plain.jsonl, $OUT/pmc/..., $OUT/summary.txt (tools/valu_peak_summary.py).
set -u
OUT=${OUT:-gpurun_out/valu_peak}
mkdir -p "$OUT"
export TMPDIR=/tmp
BIN=diag/valu_peak
[ -x $BIN ] || { echo "build $BIN first (hipcc --offload-arch=gfx950 -O3 -o $BIN diag/valu_peak.hip)"; exit 2; }
echo "== plain"
timeout -k 10 180 ./$BIN > "$OUT/plain.jsonl" 2> "$OUT/plain.err"
rc=$?; echo "   rc=$rc"; cat "$OUT/plain.err"
[ $rc = 0 ] || exit $rc
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
echo "== pmc $CTRS"
timeout -s KILL 180 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/pmc" -o pmc -- ./$BIN > "$OUT/pmc.jsonl" 2> "$OUT/pmc.err"
rc=$?; echo "   rc=$rc"; tail -n 3 "$OUT/pmc.err"
[ $rc = 0 ] || exit $rc
python tools/valu_peak_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
