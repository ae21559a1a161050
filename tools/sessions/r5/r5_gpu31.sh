#!/bin/bash
# Round 5 DIAGNOSTIC: per-wave stamps of the C2 fused step and tail, N = 1 and rank 3 of 8 (build/rtw_wstamps.so)
set -u
OUT=gpurun_out/r5/wstamps; mkdir -p $OUT
RTW_LIB=build/rtw_wstamps.so timeout -k 10 300 python diag/run_wave_stamps.py 1 0 $OUT/n1.json > $OUT/n1.log 2>&1 || { tail $OUT/n1.log; exit 1; }
cat $OUT/n1.log | grep -v amdgpu.ids
RTW_LIB=build/rtw_wstamps.so timeout -k 10 300 python diag/run_wave_stamps.py 8 3 $OUT/r3.json > $OUT/r3.log 2>&1 || { tail $OUT/r3.log; exit 1; }
cat $OUT/r3.log | grep -v amdgpu.ids
