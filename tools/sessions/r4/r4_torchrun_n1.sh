#!/bin/bash
# bench.py's driver-shaped multi-GPU launch at N = 1 on the box (torch.distributed.run, RCCL backend, one
# rank: shard render, dist.gather, reassembly, barrier + max-over-ranks timing) and the single-process
# rtw_multi path at N = 1; lines under gpurun_out/tr/.
set -u
OUT=gpurun_out/tr
mkdir -p "$OUT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/torchrun_n1.json" 2> "$OUT/torchrun_n1.err" || { tail -20 "$OUT/torchrun_n1.err"; exit 1; }
grep "^{" "$OUT/torchrun_n1.json" | tail -1 | cut -c1-400
timeout -k 10 300 python bench.py --gpus 1 --single-process --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/single_n1.json" 2> "$OUT/single_n1.err" || { tail -20 "$OUT/single_n1.err"; exit 1; }
grep "^{" "$OUT/single_n1.json" | tail -1 | cut -c1-400
