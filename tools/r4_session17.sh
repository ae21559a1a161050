#!/bin/bash
# Round-4 session 17: the final measurement of the in-tree build (tools/r4_final2.sh), then the GPU suite on
# build/rtw_rng.so (RNG state in the 60-B layout's spare ray words) and its A/B vs in-tree.
set -u
bash tools/r4_final2.sh || exit $?
bash tools/r4_session16.sh || exit $?
