# A/B (same box, alternating, 2 reps): product build vs build/rtw_ilp.so (rtw_wavefront.hip compiled with -mllvm -amdgpu-sched-strategy=max-ilp; other TUs unchanged)
set -u
mkdir -p gpurun_out/ab
for rep in 1 2; do
for lib in ${LIBS:-default build/rtw_ilp.so}; do
  for c in c2 c4 cornell; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    RTW_LIB=$L timeout -k 10 240 python bench.py --config $c --no-cpu-baseline --steps 3 > gpurun_out/ab/${c}_$(basename $lib)_$rep.json 2>/dev/null || exit $?
    python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],sys.argv[3],d['value'],d['roofline']['kernel_ms_per_step'])" gpurun_out/ab/${c}_$(basename $lib)_$rep.json $c $lib
  done
done
done
