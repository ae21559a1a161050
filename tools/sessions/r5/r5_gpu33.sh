#!/bin/bash
# Round 5: the driver's launch shapes at N = 1 on the final build (torchrun one rank; rtw_multi single process)
set -u
OUT=gpurun_out/r5/torchrun_n1; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --steps 3 --warmup 1 > $OUT/torchrun.json 2> $OUT/torchrun.err || { tail $OUT/torchrun.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --single-process --steps 3 --warmup 1 > $OUT/single.json 2> $OUT/single.err || { tail $OUT/single.err; exit 1; }
for f in torchrun single; do
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['n_gpus'], d['config'].get('parallelism'), r['frac'], r['hbm']['frac'])" $OUT/$f.json $f
done
