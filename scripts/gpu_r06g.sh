set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r06g_tests.log; exit 1; }
tail -2 gpurun_out/r06g_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-steps 0 > gpurun_out/r06g_b.json 2>gpurun_out/r06g_b.err || { tail -5 gpurun_out/r06g_b.err; exit 7; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r06g_b.json').read().strip().splitlines()[-1]); print('package', round(d['ms_per_step'],3), d['verified']['sample_bitexact_vs_oracle'], d['verified']['indptr_ok'], d['verified']['columns_ok'])"
done
bash scripts/gpu_kstats.sh > gpurun_out/r06g_kstats.txt 2>&1; cat gpurun_out/r06g_kstats.txt
