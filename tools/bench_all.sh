# bench.py over the BASELINE configs that fit one GPU + the §8f object scenes (one JSON line each)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 1 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
for c in c4 c5 cornell cornell_smoke simple_light; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 2 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
done
for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['hbm']['frac'], r['kernel_ms_per_step'])" gpurun_out/bench_$c.json $c
done
