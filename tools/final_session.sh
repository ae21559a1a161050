#!/bin/bash
# The end-of-round measurement session: ONE build, each part on one box (PART=pmc | bench | extra), output under
# $O (default gpurun_out/final/), copied into profiles/ by `R=<round tag> bash tools/collect_final.sh <part>` afterwards.
#   pmc:   VALU (SQ) and HBM-traffic PMC passes of bench.py for every config + the per-rank shard passes of C2 at
#          N = 2, 4, 8 (rank 0), each stamped with rtw_build_id; copied into profiles/ on the box so that
#   bench: the walk ceiling, then bench lines of every config (their rooflines from this build's passes), the C2
#          rocprofv3 --kernel-trace --stats summary;
#   extra: C2 and C4 stall passes, the C2 shard predictions at N = 1, 2, 4, 8 (tools/shard_sim.py).
set -u
O=${O:-gpurun_out/final}
mkdir -p "$O"
export TMPDIR=/tmp
PART=${PART:-pmc}
CFGS=${CFGS:-"c2 c3 c4 c5 cornell cornell_smoke simple_light"}
if [ "$PART" = pmc ]; then
  for c in $CFGS; do
    OUT=$O/pmc_$c/valu BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_valu.sh > "$O/pmc_${c}_valu.txt" 2>&1 || { tail "$O/pmc_${c}_valu.txt"; exit 1; }
    OUT=$O/pmc_$c/traffic BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_traffic.sh > "$O/pmc_${c}_traffic.txt" 2>&1 || { tail "$O/pmc_${c}_traffic.txt"; exit 1; }
    cp "$O/pmc_$c/valu/pmc_valu.json" "$O/pmc_valu_${c}_sah.json" && cp "$O/pmc_$c/traffic/pmc_traffic.json" "$O/pmc_traffic_${c}_sah.json" || exit 1
    echo "pmc $c: $(grep '^build' "$O/pmc_$c/valu/summary.txt") / $(grep '^build' "$O/pmc_$c/traffic/summary.txt")"
  done
  for n in ${SHARD_NS-2 4 8}; do
    bash tools/pmc_shard.sh c2 $n 0 > "$O/pmc_shard_n$n.txt" 2>&1 || { tail "$O/pmc_shard_n$n.txt"; exit 1; }
    cp profiles/pmc_valu_c2_sah_n${n}_r0.json profiles/pmc_traffic_c2_sah_n${n}_r0.json "$O/" || exit 1
    echo "shard pass n$n done"
  done
  exit 0
fi
if [ "$PART" = bench ]; then
  # this build's passes (from PART=pmc, already in profiles/ via collect) must be in place
  RTW_LIB=build/rtw_trav.so timeout -k 10 300 python diag/run_walk_ceiling.py c2 "$O/walk_ceiling_c2.json" > "$O/walk_c2.log" 2>&1 || { tail "$O/walk_c2.log"; exit 1; }
  cat "$O/walk_c2.log" | grep '^{'
  cp "$O/walk_ceiling_c2.json" profiles/walk_ceiling_c2.json || exit 1
  timeout -k 10 300 python bench.py > "$O/c2_bench.json" 2> "$O/c2.err" || { tail "$O/c2.err"; exit 1; }
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 1 > "$O/c3_bench.json" 2> "$O/c3.err" || { tail "$O/c3.err"; exit 1; }
  for c in c4 c5 cornell cornell_smoke simple_light; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 2 > "$O/${c}_bench.json" 2> "$O/$c.err" || { tail "$O/$c.err"; exit 1; }
  done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 0 > "$O/rocprof.log" 2>&1 || { tail "$O/rocprof.log"; exit 1; }
  grep "^{" "$O/rocprof.log" > "$O/rocprof_bench.json"
  python tools/prof_summary.py "$O"/prof/*/run_kernel_trace.csv --json "$O/rocprof_bench.json" > "$O/c2_timed_summary.txt" 2>&1 || \
    python tools/prof_summary.py "$O"/prof/run_kernel_trace.csv --json "$O/rocprof_bench.json" > "$O/c2_timed_summary.txt" 2>&1
  cp "$O"/prof/*run_kernel_stats.csv "$O/c2_kernel_stats.csv" 2>/dev/null || cp "$O"/prof/*/run_kernel_stats.csv "$O/c2_kernel_stats.csv" 2>/dev/null
  for c in $CFGS; do
    python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['valu']['issue_busy'], r['hbm']['frac'], (r.get('walk') or {}).get('frac'), r['kernel_ms_per_step'])" "$O/${c}_bench.json" $c
  done
  cat "$O/c2_timed_summary.txt" | head -30
  exit 0
fi
if [ "$PART" = extra ]; then
  bash tools/r5_c4_stall.sh c2 $O/stall_c2 > "$O/stall_c2.txt" 2>&1 || { tail "$O/stall_c2.txt"; exit 1; }
  bash tools/r5_c4_stall.sh c4 $O/stall_c4 > "$O/stall_c4.txt" 2>&1 || { tail "$O/stall_c4.txt"; exit 1; }
  timeout -k 10 600 python tools/shard_sim.py c2 > "$O/c2_shard_sim.jsonl" 2> "$O/shard_sim.err" || { tail "$O/shard_sim.err"; exit 1; }
  cat "$O/c2_shard_sim.jsonl"
  exit 0
fi
echo "unknown PART=$PART"; exit 2
