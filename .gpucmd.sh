set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
TUNE_ROUNDS=3 TUNE='[{}]' timeout -k 10 400 python tools/tune.py 100 c2 > gpurun_out/tune_c2.log 2>&1 || exit $?
TUNE_ROUNDS=2 TUNE='[{}]' timeout -k 10 400 python tools/tune.py 32 c4 > gpurun_out/tune_c4.log 2>&1 || exit $?
cat gpurun_out/tune_c2.log gpurun_out/tune_c4.log | grep '^{'
