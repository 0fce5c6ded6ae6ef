set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py tests/test_gpu_longrow.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06k_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r06k_tests.log; exit 1; }
tail -2 gpurun_out/r06k_tests.log
BENCH="--config cfg4 --steps 3 --warmup 1" bash scripts/gpu_kstats.sh > gpurun_out/r06k_kstats.txt 2>&1; cat gpurun_out/r06k_kstats.txt
timeout -k 10 600 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06k_cfg4.json 2> gpurun_out/r06k_cfg4.err || { tail -5 gpurun_out/r06k_cfg4.err; exit 7; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06k_cfg4.json').read().strip().splitlines()[-1]); print('cfg4', round(d['ms_per_step'],2), d['roofline']['frac'], d['verified'])"
