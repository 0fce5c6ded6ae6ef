set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06t_tests.log 2>&1 || { tail -30 gpurun_out/r06t_tests.log; exit 5; }
tail -2 gpurun_out/r06t_tests.log
LIBS="abvar/head.so abvar/pgate.so" bash scripts/gpu_kstats.sh > gpurun_out/r06t_kstats.txt 2>&1 || { cat gpurun_out/r06t_kstats.txt; exit 6; }
grep "==\|copy\|partition\|gather\|wave" gpurun_out/r06t_kstats.txt
for f in 1 2 3; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/ks_$f.json').read().strip().splitlines()[-1]); print($f, d['ms_per_step'], d['value'])"; done
