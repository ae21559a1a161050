# DIAGNOSTIC: bench.py per-kernel times over env settings; SWEEP = list of "VAR=val,VAR=val" (or "-")
for cfg in ${SWEEP:-"-"}; do
  envs=""
  [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/sweep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep.json')); r=d['roofline']; print('$cfg', d['value'], r['kernel_ms_per_step'])"
done
