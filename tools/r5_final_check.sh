#!/bin/bash
# Round 5: the round-end commands on the final tree -- GPU suite, smoke(), the default bench line
set -u
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f/gpu_tests_final.txt 2>&1
rc=$?; tail -3 gpurun_out/r5f/gpu_tests_final.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.txt 2>&1 || { tail gpurun_out/r5f/smoke.txt; exit 1; }
tail -3 gpurun_out/r5f/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r5f/bench_default.json 2> gpurun_out/r5f/bench_default.err || { tail gpurun_out/r5f/bench_default.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/r5f/bench_default.json') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'], r['frac'], r['hbm']['frac'], r['walk']['frac'], d['cpu_baseline']['value'])"
