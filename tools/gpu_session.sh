#!/bin/bash
# One GPU-box session: tests -> smoke -> bench -> rocprof kernel trace.
# Each GPU step has its own time limit; a crash/timeout/abort stops the script
# (plain test failures, exit 1, do not).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
  case $rc in 0|1) return 0;; *) echo "!! $name ended with $rc: stopping"; exit $rc;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -n "${TUNE_ARGS:-}" ]; then step tune 600 python tools/tune.py ${TUNE_ARGS}; fi
step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 0 ${BENCH_ARGS:-}
  grep "^{" "$OUT/rocprof.log" > "$OUT/rocprof_bench.json" || true
  python tools/prof_summary.py "$OUT/prof/run_kernel_trace.csv" --json "$OUT/rocprof_bench.json" > "$OUT/prof_timed_summary.txt" 2>&1 || true
  cat "$OUT/prof_timed_summary.txt"
fi
if [ "${PMC:-0}" = 1 ]; then
  step pmc 1300 bash tools/pmc_traffic.sh
fi
echo "== done $(date +%T)"
