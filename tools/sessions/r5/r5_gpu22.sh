#!/bin/bash
# Round 5: default deal 59 -- whole GPU suite, bench lines, the C2 8-rank breakdown and a per-launch trace of rank 3
set -u
bash tools/sessions/r5/r5_gpu9.sh || exit 1
TAG=deal59 bash tools/r5_shard_breakdown.sh c2 8 || exit 1
TAG=deal59 bash tools/r5_shard_trace.sh 8 3 || exit 1
