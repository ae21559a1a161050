#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (MI355X_MICROARCH.md § HBM):
# FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots); kernel-trace only.
# Output: gpurun_out/pmc_traffic/{fetch,write}/... and pmc_traffic.json (tools/pmc_summary.py).
set -u
OUT=${OUT:-gpurun_out/pmc_traffic}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 1 --warmup 0"}
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== $c"
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/$c" -o pmc -- python bench.py $ARGS > "$OUT/$c.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 1 "$OUT/$c.log" | cut -c1-200
  case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
done
python tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
