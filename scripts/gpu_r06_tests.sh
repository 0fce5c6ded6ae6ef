set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06_gpu_tests.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06_gpu_tests.log | grep -v PASSED | head -20
exit $rc
