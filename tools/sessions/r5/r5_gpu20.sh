#!/bin/bash
# Round 5: deal 51 (1|2|16|32) on the other configs, and dynamic dealing forced on small batches (bit 8: 59 / 57)
# for one rank's shard of 8 and simple_light
set -u
mkdir -p gpurun_out/r5
OUT=gpurun_out/r5/ab_deal6_c2_r3 BENCH_EXTRA="--shard 8,3" CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"deal": 51}' '{"deal": 59}' '{"deal": 57}' || exit 1
OUT=gpurun_out/r5/ab_deal6_simple_light CONFIG=simple_light ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"deal": 51}' '{"deal": 59}' '{"deal": 57}' || exit 1
for cfg in c5 cornell_smoke c3; do
  st=3; [ $cfg = c3 ] && st=1
  OUT=gpurun_out/r5/ab_deal6_$cfg CONFIG=$cfg ROUNDS=2 STEPS=$st bash tools/ab_knob.sh '' '{"deal": 51}' || exit 1
done
