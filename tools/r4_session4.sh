#!/bin/bash
# Round-4 session 4: C4 traffic and L2 hit counters of the in-tree (packed-state) library and build/rtw_head.so,
# per kernel (why the packed layout's trace is slower on C4 while its shade is faster).
set -u
export TMPDIR=/tmp
OUT0=gpurun_out/s4
mkdir -p "$OUT0"
for lib in "" build/rtw_head.so; do
  tag=$(basename "${lib:-default}" .so)
  RTW_LIB=$lib OUT=$OUT0/traffic_$tag BENCH_ARGS="--config c4 --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_traffic.sh > "$OUT0/traffic_$tag.txt" 2>&1 || { cat "$OUT0/traffic_$tag.txt"; exit 1; }
  RTW_LIB=$lib timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $OUT0/cache_$tag -o pmc -- python bench.py --config c4 --no-cpu-baseline --steps 1 --warmup 0 > $OUT0/cache_$tag.log 2>&1 || exit $?
  echo "$tag done"
done
