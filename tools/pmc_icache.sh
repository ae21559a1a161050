#!/bin/bash
# Instruction-cache counters of one render per config (two SQC counters + SQ_IFETCH per pass,
# kernel-trace only; each pass under its own kill timeout).  Output: gpurun_out/pmc_icache/<config>/
set -u
OUT=${OUT:-gpurun_out/pmc_icache}
export TMPDIR=/tmp
for cfg in ${CONFIGS:-cornell c2}; do
  mkdir -p "$OUT/$cfg"
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU --kernel-trace \
    --output-format csv -d "$OUT/$cfg" -o pmc -- python tools/render_once.py $cfg ${SPP:-16} > "$OUT/$cfg/run.log" 2>&1
  rc=$?
  echo "$cfg rc=$rc"; tail -n 2 "$OUT/$cfg/run.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    print(f)
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0))[:6]:
        h, m = v.get("SQC_ICACHE_HITS", 0), v.get("SQC_ICACHE_MISSES", 0)
        print(f"  {k:60s} icache hit rate {h / max(1, h + m):.4f}  misses {m:.4g}  ifetch {v.get('SQ_IFETCH', 0):.4g}  "
              f"valu {v.get('SQ_INSTS_VALU', 0):.4g}")
PY
