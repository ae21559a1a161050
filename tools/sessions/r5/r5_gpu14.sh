#!/bin/bash
# Round 5: strong-scaling prediction on the current defaults (4-copy stage, 2 x 768, deal 3, balanced rows)
set -u
TAG=final1 bash tools/r5_shard_breakdown.sh c2 8 || exit 1
TAG=final1 bash tools/r5_shard_breakdown.sh c2 4 || exit 1
TAG=final1 bash tools/r5_shard_breakdown.sh c2 2 || exit 1
