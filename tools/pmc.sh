#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) on the tuning workload.
set -u
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
SPP=${SPP:-20}
CFG=${CFG:-c2}
export TUNE=${TUNE:-'[{"kernel": 1}]'}
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
fi
i=0
for grp in ${GROUPS_:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
             "SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAIT_INST_LDS" \
             "SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,GRBM_GUI_ACTIVE" \
             "SQ_THREAD_CYCLES_VALU,SQ_INST_CYCLES_VMEM,SQ_INSTS_SMEM,SQ_INSTS_BRANCH" \
             "FETCH_SIZE" "WRITE_SIZE"}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc -- python tools/tune.py $SPP $CFG > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 2 "$OUT/p$i.log"
  case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
done
