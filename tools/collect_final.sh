#!/bin/bash
# Copy a tools/final_session.sh session ($O, default gpurun_out/final/) into profiles/ under the round tag R
# (run here, after the gpurun call).
# usage: R=r6 bash tools/collect_final.sh pmc|bench|extra
set -eu
O=${O:-gpurun_out/final}
R=${R:?set R, the round tag (e.g. r6)}
case ${1:-} in
  pmc)
    cp $O/pmc_valu_*_sah*.json $O/pmc_traffic_*_sah*.json profiles/
    mkdir -p profiles/${R}_pmc
    for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do
      cp $O/pmc_$c/valu/summary.txt profiles/${R}_pmc/${c}_valu_summary.txt
      cp $O/pmc_$c/traffic/summary.txt profiles/${R}_pmc/${c}_traffic_summary.txt
    done ;;
  bench)
    for c in c2 c3 c4 c5 cornell cornell_smoke simple_light; do cp $O/${c}_bench.json profiles/${R}_${c}_bench.json; done
    cp $O/walk_ceiling_c2.json profiles/walk_ceiling_c2.json
    cp $O/c2_timed_summary.txt profiles/${R}_c2_timed_summary.txt
    cp $O/c2_kernel_stats.csv profiles/${R}_c2_kernel_stats.csv ;;
  extra)
    mkdir -p profiles/${R}_stall
    for c in c2 c4; do
      cp $O/stall_$c/summary.txt profiles/${R}_stall/${c}_summary.txt
      cp $O/stall_$c/pmc_stall.json profiles/${R}_stall/${c}_pmc_stall.json
      cp $O/stall_$c/cache/summary.txt profiles/${R}_stall/${c}_cache_summary.txt
    done
    cp $O/c2_shard_sim.jsonl profiles/${R}_c2_shard_sim.jsonl ;;
  *) echo "usage: $0 pmc|bench|extra"; exit 2 ;;
esac
