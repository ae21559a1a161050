# Round 4: (1) the C5 / simple_light question of VERDICT r3 item 7 -- the library at 722d11e against the
# round-3 final 4484266, three alternating rounds on one box; (2) C3's shard prediction at 1/2/4/8 ranks;
# (3) C4 with the fused step through L1/L2 (fuse 7) against the split kernels.
set -o pipefail
mkdir -p gpurun_out/r4_c5sl
for c in c5 simple_light; do
  OUT=gpurun_out/r4_c5sl CONFIG=$c ROUNDS=3 STEPS=3 bash tools/ab_c2.sh build/rtw_722d11e.so build/rtw_4484266.so || exit $?
done
timeout -k 10 300 python tools/shard_sim.py c3 0 8 1,2,4,8 > gpurun_out/r4_c3_shard_sim.jsonl 2> gpurun_out/r4_c3_shard_sim.err || exit $?
cat gpurun_out/r4_c3_shard_sim.jsonl
OUT=gpurun_out/r4_c4fuse CONFIG=c4 ROUNDS=2 STEPS=3 bash tools/ab_knob.sh "" '{"fuse": 7}' || exit $?
