set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r06h_tests.log; exit 1; }
tail -2 gpurun_out/r06h_tests.log
LIBS="abvar/w8.so" ROUNDS=2 bash scripts/gpu_ab.sh
LIBS="abvar/w8.so" bash scripts/gpu_kstats.sh > gpurun_out/r06h_kstats.txt 2>&1; grep "==\|wave\|gather\|partition\|copy" gpurun_out/r06h_kstats.txt
