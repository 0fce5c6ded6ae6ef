set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_staged.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err && tail -c 600 gpurun_out/r06a_bench.json
timeout -k 10 400 python bench.py --dist powerlaw --steps 20 --warmup 5 --host-steps 3 --no-cpu-baseline > gpurun_out/r06a_bench_powerlaw.json 2> gpurun_out/r06a_bench_powerlaw.err && tail -c 300 gpurun_out/r06a_bench_powerlaw.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --call async --host-steps 0 --no-cpu-baseline > gpurun_out/r06a_bench_async.json 2> gpurun_out/r06a_bench_async.err
