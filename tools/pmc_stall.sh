#!/bin/bash
# Stall breakdown of the bench's kernels per launch: SQ counter groups, one
# rocprofv3 --pmc pass each (<= 8 SQ counters per pass, kernel-trace only), over
# `bench.py --steps 1 --warmup 0` of $BENCH_ARGS.  Summary: tools/pmc_stall_summary.py.
set -u
OUT=${OUT:-gpurun_out/pmc_stall}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 1 --warmup 0"}
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM"
G3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
G4="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_IFETCH"
i=0
# GROUPS_PMC_<k> unset: the default group; set but empty: the group is skipped
for grp in "${GROUPS_PMC_1-$G1}" "${GROUPS_PMC_2-$G2}" "${GROUPS_PMC_3-$G3}" "${GROUPS_PMC_4-$G4}"; do
  i=$((i + 1))
  [ -n "$grp" ] || continue
  echo "== g$i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o pmc -- python bench.py $ARGS > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 2 "$OUT/g$i.log" | cut -c1-300
  # 1 = rocprofv3 refused the counter set (unknown counter): next group; anything else stops
  case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
done
python tools/pmc_stall_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
