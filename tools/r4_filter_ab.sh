# Same-box A/B of the in-tree library against ${PREV:-build/rtw_head.so} (the build before a kernel change):
# GPU tests first (the change must keep every image), then C2 twice and the other configs once.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_ab.txt 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_ab.txt; [ $rc = 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} STEPS=5 bash tools/ab_c2.sh "" ${PREV:-build/rtw_head.so} || exit $?
for c in ${CONFIGS:-c4 c5 cornell cornell_smoke simple_light}; do CONFIG=$c ROUNDS=1 STEPS=3 bash tools/ab_c2.sh "" ${PREV:-build/rtw_head.so} || exit $?; done
