set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longrow.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ab_tests.log 2>&1 || { tail -30 gpurun_out/r06ab_tests.log; exit 5; }
tail -2 gpurun_out/r06ab_tests.log
LIBS="abvar/head.so" BENCH="--config cfg4 --steps 3 --warmup 1" bash scripts/gpu_kstats.sh > gpurun_out/r06ab_kstats4.txt 2>&1 || { cat gpurun_out/r06ab_kstats4.txt; exit 7; }
cat gpurun_out/r06ab_kstats4.txt
