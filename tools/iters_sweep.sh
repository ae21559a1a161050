# DIAGNOSTIC: bench.py per-kernel times over rtw_tuning settings; SWEEP = list of JSON objects (or "-")
for cfg in ${SWEEP:-"-"}; do
  tun=""
  [ "$cfg" != "-" ] && tun="$cfg"
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --tuning "$tun" $BENCH_ARGS > gpurun_out/sweep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep.json')); r=d['roofline']; print('$cfg', d['value'], r['kernel_ms_per_step'])"
done
