#!/bin/bash
# Copy a tools/final_r5.sh session (gpurun_out/r5f/) into profiles/ (run here, after the gpurun call).
# usage: bash tools/collect_r5.sh pmc|bench|extra
set -eu
O=gpurun_out/r5f
case ${1:-} in
  pmc)
    cp $O/pmc_valu_*_sah*.json $O/pmc_traffic_*_sah*.json profiles/
    mkdir -p profiles/r5_pmc
    for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
      cp $O/pmc_$c/valu/summary.txt profiles/r5_pmc/${c}_valu_summary.txt
      cp $O/pmc_$c/traffic/summary.txt profiles/r5_pmc/${c}_traffic_summary.txt
    done ;;
  bench)
    for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do cp $O/${c}_bench.json profiles/r5_${c}_bench.json; done
    cp $O/walk_ceiling_c2.json profiles/walk_ceiling_c2.json
    cp $O/c2_timed_summary.txt profiles/r5_c2_timed_summary.txt
    cp $O/c2_kernel_stats.csv profiles/r5_c2_kernel_stats.csv ;;
  extra)
    mkdir -p profiles/r5_stall
    for c in c2 c4; do
      cp $O/stall_$c/summary.txt profiles/r5_stall/${c}_summary.txt
      cp $O/stall_$c/pmc_stall.json profiles/r5_stall/${c}_pmc_stall.json
      cp $O/stall_$c/cache/summary.txt profiles/r5_stall/${c}_cache_summary.txt
    done
    cp $O/c2_shard_sim.jsonl profiles/r5_c2_shard_sim.jsonl ;;
  *) echo "usage: $0 pmc|bench|extra"; exit 2 ;;
esac
