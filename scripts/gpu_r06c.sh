set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06c_tests.log; exit 1; }
tail -2 gpurun_out/r06c_tests.log
LIBS="abvar/g24.so abvar/g32.so abvar/g16b.so abvar/g16c.so abvar/p1g16.so abvar/p1g24.so" bash scripts/gpu_kstats.sh > gpurun_out/r06c_kstats.txt 2>&1; grep "==\|gather\|partition" gpurun_out/r06c_kstats.txt
timeout -k 10 400 python bench.py --dist powerlaw --steps 20 --warmup 5 --host-steps 3 --no-cpu-baseline > gpurun_out/r06c_bench_powerlaw.json 2> gpurun_out/r06c_bench_powerlaw.err
