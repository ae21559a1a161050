#!/bin/bash
# Round 5: does the dynamic claim of iterations >= 1 (deal bit 16) cost on small batches?  rank 3 of 8 and the full
# frame in 8 batches (wf_paths 2^26): 59 vs 43 (59 without bit 16) vs 11 (1|2|8)
set -u
mkdir -p gpurun_out/r5
OUT=gpurun_out/r5/ab_bit16_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"deal": 43}' '{"deal": 11}' || exit 1
OUT=gpurun_out/r5/ab_bit16_c2_b8 CONFIG=c2 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"wf_paths": 67108864}' '{"deal": 43, "wf_paths": 67108864}' '{"deal": 11, "wf_paths": 67108864}' || exit 1
