#!/bin/bash
# Round 5: why iteration 0 costs 19 % more with direction bucketing (C2 N = 1): VALU and traffic passes with
# sort_iters 0, to set beside the final build's default passes (profiles/r5_pmc/c2_*)
set -u
O=gpurun_out/r5/sort0_pmc; mkdir -p $O
OUT=$O/valu BENCH_ARGS='--config c2 --no-cpu-baseline --steps 1 --warmup 0 --tuning {"sort_iters":0}' bash tools/pmc_valu.sh > $O/valu.txt 2>&1 || { tail $O/valu.txt; exit 1; }
OUT=$O/traffic BENCH_ARGS='--config c2 --no-cpu-baseline --steps 1 --warmup 0 --tuning {"sort_iters":0}' bash tools/pmc_traffic.sh > $O/traffic.txt 2>&1 || { tail $O/traffic.txt; exit 1; }
head -12 $O/valu/summary.txt; cat $O/traffic/summary.txt
