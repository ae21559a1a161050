#!/bin/bash
# ISA evidence of the product kernels: registers, scratch, occupancy, instruction
# classes and the walk loops of the fused step, the L1/L2 trace, the tails and the shade kernel.
# Output: profiles/<tag>/isa_report.{txt,json}
set -eu
TAG=${1:-r3_isa}
make -s -C zig-raytracing-weekend_amd/csrc isa
mkdir -p profiles/$TAG
python tools/isa_report.py build/isa/rtw_wavefront_all.s \
  wf_step_cldsILj0E wf_traceILj0ELb0E wf_tail_cldsILj0E wf_tail_w5ILj0E wf_shadeILj0E 'wf_stepILj49ELb1E' \
  'wf_stepILj7ELb1E' --json profiles/$TAG/isa_report.json > profiles/$TAG/isa_report.txt
grep -E "^==|meta|WALK" profiles/$TAG/isa_report.txt | head -40
