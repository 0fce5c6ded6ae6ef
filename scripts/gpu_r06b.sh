set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06b_tests.log; exit 1; }
tail -2 gpurun_out/r06b_tests.log
LIBS="abvar/base.so abvar/g4.so abvar/g16.so" bash scripts/gpu_kstats.sh > gpurun_out/r06b_kstats.txt 2>&1; cat gpurun_out/r06b_kstats.txt
timeout -k 10 300 python -u scripts/probes/stream_probe.py powerlaw > gpurun_out/r06b_stream_pl.txt 2>&1; cat gpurun_out/r06b_stream_pl.txt | grep pass
