#!/bin/bash
# Round 5: per-launch stall breakdown of C4's kernels (wf_trace, wf_shade, wf_tail_w5)
# and their cache behaviour, same build, one box.
set -u
mkdir -p gpurun_out/r5
OUT=gpurun_out/r5/c4_stall BENCH_ARGS="--config c4 --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_stall.sh || exit $?
OUT=gpurun_out/r5/c4_stall GROUPS_PMC_1="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
  GROUPS_PMC_2="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" GROUPS_PMC_3="" GROUPS_PMC_4="" \
  bash -c 'OUTB=$OUT; OUT=$OUTB/cache bash tools/pmc_stall.sh' || exit $?
