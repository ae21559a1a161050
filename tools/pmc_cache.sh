set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_cache}; CFG=${CFG:-c4}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $OUT/a -o pmc -- python bench.py --config $CFG --no-cpu-baseline --steps 1 --warmup 0 > $OUT/a.log 2>&1
echo rc=$?
