#!/bin/bash
# Round-4 measurement session on ONE box and ONE build:
#   1. the VALU (SQ) and HBM-traffic (FETCH_SIZE / WRITE_SIZE) PMC passes of bench.py for every config,
#      each stamped with the library's rtw_build_id (tools/pmc_valu_summary.py, tools/pmc_summary.py);
#   2. their JSON copied into profiles/ on the box, so the bench lines of step 3 take their roofline from
#      passes of this very build (bench.py uses no pass of another build);
#   3. bench lines of every config, the C2 rocprofv3 --kernel-trace --stats summary, the C2 stall passes.
# Output under gpurun_out/r4/ (copied into profiles/ by hand afterwards).
set -u
OUT=gpurun_out/r4
mkdir -p "$OUT"
export TMPDIR=/tmp
CFGS=${CFGS:-"c2 c3 c4 c5 cornell cornell_smoke simple_light"}
if [ "${SKIP_PMC:-0}" != 1 ]; then
  for c in $CFGS; do
    OUT=$OUT/pmc_$c/valu BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_valu.sh > "$OUT/pmc_${c}_valu.txt" 2>&1 || { cat "$OUT/pmc_${c}_valu.txt"; exit 1; }
    OUT=$OUT/pmc_$c/traffic BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_traffic.sh > "$OUT/pmc_${c}_traffic.txt" 2>&1 || { cat "$OUT/pmc_${c}_traffic.txt"; exit 1; }
    cp "$OUT/pmc_$c/valu/pmc_valu.json" "profiles/pmc_valu_${c}_sah.json" || exit 1
    cp "$OUT/pmc_$c/traffic/pmc_traffic.json" "profiles/pmc_traffic_${c}_sah.json" || exit 1
    echo "pmc $c: $(grep '^build' "$OUT/pmc_$c/valu/summary.txt") / $(grep '^build' "$OUT/pmc_$c/traffic/summary.txt")"
  done
fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 300 python bench.py > "$OUT/c2_bench.json" 2> "$OUT/c2.err" || exit $?
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 1 > "$OUT/c3_bench.json" 2> "$OUT/c3.err" || exit $?
for c in c4 c5 cornell cornell_smoke simple_light; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 2 > "$OUT/${c}_bench.json" 2> "$OUT/$c.err" || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 0 > "$OUT/rocprof.log" 2>&1 || exit $?
grep "^{" "$OUT/rocprof.log" > "$OUT/rocprof_bench.json"
python tools/prof_summary.py "$OUT"/prof/*/run_kernel_trace.csv --json "$OUT/rocprof_bench.json" > "$OUT/c2_timed_summary.txt" 2>&1 || \
  python tools/prof_summary.py "$OUT"/prof/run_kernel_trace.csv --json "$OUT/rocprof_bench.json" > "$OUT/c2_timed_summary.txt" 2>&1
cp "$OUT"/prof/*run_kernel_stats.csv "$OUT/c2_kernel_stats.csv" 2>/dev/null || cp "$OUT"/prof/*/run_kernel_stats.csv "$OUT/c2_kernel_stats.csv" 2>/dev/null
if [ "${STALL:-1}" = 1 ]; then
  OUT=$OUT/stall_c2 bash tools/pmc_stall.sh > "$OUT/stall_c2.txt" 2>&1 || exit $?
fi
for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['valu']['issue_busy'], r['hbm']['frac'], r['kernel_ms_per_step'])" "$OUT/${c}_bench.json" $c
done
cat "$OUT/c2_timed_summary.txt"
