#!/bin/bash
# Round 5: 8-rank prediction vs wavefront iterations before the tail (6 / 7 / 8 / 9)
set -u
for it in 6 7 8; do TAG=it$it bash tools/r5_shard_breakdown.sh c2 8 "{\"wf_iters\": $it}" || exit 1; done
