set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || { tail -5 gpurun_out/r06c_bench.err; exit 4; }
tail -c 300 gpurun_out/r06c_bench.json; echo
timeout -k 10 400 python -u bench.py --dist powerlaw --steps 20 --warmup 5 --host-steps 3 --no-cpu-baseline > gpurun_out/r06c_bench_powerlaw.json 2> gpurun_out/r06c_bench_powerlaw.err || { tail -5 gpurun_out/r06c_bench_powerlaw.err; exit 5; }
timeout -k 10 400 python -u bench.py --config kdd9x --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06c_bench_kdd9x.json 2> gpurun_out/r06c_bench_kdd9x.err || { tail -5 gpurun_out/r06c_bench_kdd9x.err; exit 6; }
timeout -k 10 400 python -u bench.py --boundary libsvm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06c_bench_libsvm.json 2> gpurun_out/r06c_bench_libsvm.err || { tail -5 gpurun_out/r06c_bench_libsvm.err; exit 7; }
echo bench-done
timeout -k 10 600 python -u bench.py --config cfg4 --steps 5 --warmup 2 > gpurun_out/r06c_bench_cfg4.json 2> gpurun_out/r06c_bench_cfg4.err || { tail -5 gpurun_out/r06c_bench_cfg4.err; exit 8; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r06c_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06c_gpu_tests.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06c_gpu_tests.log | grep -v PASSED | head -20
exit $rc
