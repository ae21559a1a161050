#!/bin/bash
# SQ issue counters of the wavefront kernels (one rocprofv3 --pmc pass per group,
# kernel-trace only), over a short tools/tune.py render of BASELINE config 2.
# Output: gpurun_out/pmc_sq/<group>/... and summary.txt (tools/pmc_sq_summary.py).
set -u
OUT=${OUT:-gpurun_out/pmc_sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
SPP=${SPP:-10}
DEFAULT_SET='[{}]'
TUNE_SET=${TUNE_SET:-$DEFAULT_SET}
i=0
DEFAULT_GROUPS="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAVES,SQ_BUSY_CYCLES"
for g in ${GROUPS_PMC:-$DEFAULT_GROUPS}; do
  grp=$(echo "$g" | tr ',' ' ')
  i=$((i + 1))
  echo "== $grp"
  TUNE="$TUNE_SET" timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o pmc -- python tools/tune.py $SPP c2 > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 2 "$OUT/g$i.log" | cut -c1-300
  # 1 = rocprofv3 refused the counter set (unknown counter): try the next group; anything else stops
  case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
done
python tools/pmc_sq_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
