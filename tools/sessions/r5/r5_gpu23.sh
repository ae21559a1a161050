#!/bin/bash
# Round 5: is iteration 1's excess on a shard (rank 3 of 8: +23 % over 1/8 of N = 1) the coherent queues' padding?
# sort_iters / sort_bits on the shard and on the whole frame
set -u
mkdir -p gpurun_out/r5
OUT=gpurun_out/r5/ab_sort_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"sort_iters": 1}' '{"sort_iters": 2}' '{"sort_bits": 2}' '{"sort_iters": 0}' || exit 1
OUT=gpurun_out/r5/ab_sort_c2 CONFIG=c2 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '' '{"sort_iters": 1}' '{"sort_iters": 2}' '{"sort_bits": 2}' || exit 1
