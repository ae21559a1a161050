#!/bin/bash
# Single-process rtw_multi at N = 1 (one device: communicator, self send/recv, pack/unpack all run)
# against the single-context bench, in one box session, plus a rocprofv3 kernel trace of the multi
# path (where its overhead goes).  Results under $OUT.
set -u
OUT=${OUT:-gpurun_out/multi_n1}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "!! $name ended with $rc: stopping"; exit $rc; }
}
for rep in 1 2; do
  run single_$rep 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
  run multi_$rep 300 python bench.py --gpus 1 --single-process --steps 10 --warmup 2 --no-cpu-baseline
done
run rocprof_multi 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o multi --output-format csv -- \
    python bench.py --gpus 1 --single-process --steps 3 --warmup 1 --no-cpu-baseline
echo "== done $(date +%T)"
