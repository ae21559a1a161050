#!/bin/bash
# Timing-only ablation builds of the wavefront kernels (wrong images by construction; never the product):
# rtw_wavefront.hip recompiled with each -D flag and linked with the product's other objects.
# usage: bash tools/ablate_wf.sh RTW_ABLATE_WALK2 RTW_ABLATE_REJECT ...  -> build/rtw_<flag>.so
set -eu
cd "$(dirname "$0")/../zig-raytracing-weekend_amd/csrc"
make -s -j8 > /dev/null
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics"
OBJS="obj/rtw_host.o obj/rtw_bvh.o obj/rtw_kernels.o obj/rtw_output.o obj/rtw_multi.o obj/rtw_cpu.o"
for d in "$@"; do
  tag=$(echo "$d" | tr 'A-Z' 'a-z' | sed 's/^rtw_//')
  ( /opt/rocm/bin/hipcc $F -D$d -c -o /tmp/wf_$tag.o rtw_wavefront.hip &&
    /opt/rocm/bin/hipcc $F -shared -o ../../build/rtw_$tag.so $OBJS /tmp/wf_$tag.o -L/opt/rocm/lib -lrccl \
      -Wl,-rpath,/opt/rocm/lib -pthread && echo "built build/rtw_$tag.so" ) &
done
wait
