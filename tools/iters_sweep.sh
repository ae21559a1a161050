# DIAGNOSTIC: bench.py per-kernel times over wavefront knobs (env pairs "ITERS:PATHS")
for cfg in ${SWEEP:-"6:67108864 9:67108864 12:67108864"}; do
  it=${cfg%%:*}; paths=${cfg##*:}
  RTW_WF_ITERS=$it RTW_WF_PATHS=$paths timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_$it_$paths.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep_$it_$paths.json')); r=d['roofline']; print('$it', '$paths', d['value'], r['kernel_ms_per_step'])"
done
