set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config cfg4 --steps 5 --warmup 2 > gpurun_out/r06b_bench_cfg4.json 2> gpurun_out/r06b_bench_cfg4.err || { tail -5 gpurun_out/r06b_bench_cfg4.err; exit 4; }
tail -c 300 gpurun_out/r06b_bench_cfg4.json; echo
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r06b_gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06b_gpu_tests.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06b_gpu_tests.log | grep -v PASSED | head -20
exit $rc
