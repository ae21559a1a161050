#!/bin/bash
# Round 5: the whole GPU suite on the new defaults (deal 1), then one bench line per config (no CPU leg).
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/gpu9_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu9_tests.txt; [ $rc = 0 ] || exit $rc
for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
  st=3; [ $c = c3 ] && st=1
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps $st > gpurun_out/r5/b9_$c.json 2> gpurun_out/r5/b9.err || { tail gpurun_out/r5/b9.err; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'])" gpurun_out/r5/b9_$c.json $c
done
