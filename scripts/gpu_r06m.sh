set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r06m_tests.log; exit 1; }
tail -2 gpurun_out/r06m_tests.log
LIBS="abvar/head2.so" ROUNDS=3 BENCH="--dist powerlaw" bash scripts/gpu_ab.sh
