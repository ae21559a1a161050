#!/bin/bash
# Round 5: 8 direction buckets (sort_bits 3) instead of 16 on the large batches (C2, C5, C3)
set -u
for cfg in c2 c5; do
  st=3; [ $cfg = c5 ] && st=2
  OUT=gpurun_out/r5/ab_sortbits3_$cfg CONFIG=$cfg ROUNDS=2 STEPS=$st bash tools/ab_knob.sh '' '{"sort_bits": 3}' || exit 1
done
