#!/bin/bash
# Round-3 bench lines of every config (bench.py with the current PMC profiles) + the C2 rocprof timed summary.
# Output: gpurun_out/r3/<config>_bench.json, gpurun_out/r3/c2_timed_summary.txt
set -u
OUT=gpurun_out/r3
mkdir -p "$OUT"
export TMPDIR=/tmp
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
for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['hbm']['frac'], r['kernel_ms_per_step'])" "$OUT/${c}_bench.json" $c
done
cat "$OUT/c2_timed_summary.txt"
