#!/bin/bash
# Per-iteration kernel times of one render under each tuning (rocprofv3 kernel trace + tools/iter_times.py).
# usage: CONFIG=c4 SPP=64 bash tools/iter_ab.sh '' '{"sort_iters": 0}'
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/it}
mkdir -p "$OUT"
CONFIG=${CONFIG:-c4}; SPP=${SPP:-64}
n=0
for tu in "$@"; do
  n=$((n+1))
  rm -rf "$OUT/p$n"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/p$n" -o run --output-format csv -- \
    python3 tools/render_once.py $CONFIG $SPP ${tu:+"$tu"} > "$OUT/p$n.log" 2>&1 || { echo "render '$tu' failed"; tail -5 "$OUT/p$n.log"; exit 1; }
  f=$(ls "$OUT"/p$n/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(ls "$OUT"/p$n/run_kernel_trace.csv)
  python3 tools/iter_times.py "$f" "$CONFIG $tu" | tee -a "$OUT/iter_times.jsonl"
done
