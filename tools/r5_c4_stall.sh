#!/bin/bash
# Round 5: per-launch stall breakdown of C4's kernels (wf_trace, wf_shade, wf_tail) and their
# cache behaviour, same build, one box.  usage: bash tools/r5_c4_stall.sh [config] [out]
set -u
CFG=${1:-c4}; O=${2:-gpurun_out/r5/${CFG}_stall}
mkdir -p gpurun_out/r5
export BENCH_ARGS="--config $CFG --no-cpu-baseline --steps 1 --warmup 0"
OUT=$O bash tools/pmc_stall.sh || exit $?
OUT=$O/cache GROUPS_PMC_1="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
  GROUPS_PMC_2="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" GROUPS_PMC_3="" GROUPS_PMC_4="" \
  bash tools/pmc_stall.sh || exit $?
