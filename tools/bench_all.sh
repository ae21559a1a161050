# bench.py over the BASELINE configs that fit one GPU + the §8f object scenes (one JSON line each)
set -u
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
for c in c4 c5 cornell cornell_smoke simple_light; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 2 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
done
