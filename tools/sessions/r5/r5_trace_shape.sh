#!/bin/bash
# kernel trace (grid, workgroup, LDS, VGPR per dispatch) of one C2 render under a tuning
set -u
TU=${1:-'{"bvh_orders": 4}'}; TAG=${2:-y4}
mkdir -p gpurun_out/r5/shape_$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/shape_$TAG -o kt -- \
  python bench.py --config c2 --spp 64 --no-cpu-baseline --steps 1 --warmup 0 --tuning "$TU" > gpurun_out/r5/shape_$TAG/bench.log 2>&1
rc=$?; tail -c 300 gpurun_out/r5/shape_$TAG/bench.log; exit $rc
