set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_staged.py -x -q --timeout 200 --timeout-method thread -k "rowlane" > gpurun_out/r06q_tests.log 2>&1 || { tail -30 gpurun_out/r06q_tests.log; exit 5; }
tail -2 gpurun_out/r06q_tests.log
LIBS="${LIBS:-abvar/head.so}" bash scripts/gpu_kstats.sh > gpurun_out/r06q_kstats.txt 2>&1 || { cat gpurun_out/r06q_kstats.txt; exit 6; }
grep "==\|copy\|wave" gpurun_out/r06q_kstats.txt
BA="--steps 1 --warmup 0 --no-cpu-baseline --host-steps 0"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -T --output-format csv -d gpurun_out/r06q_ic_1 -o pmc -- python3 bench.py $BA > gpurun_out/r06q_ic_1.log 2>&1 || { tail -5 gpurun_out/r06q_ic_1.log; exit 7; }
python3 scripts/pmc_kernels.py gpurun_out/r06q_ic > gpurun_out/r06q_ic.json && python3 -c "
import json; d=json.load(open('gpurun_out/r06q_ic.json'))
for k,v in d.items():
    if 'lpr_' in k: print(k[-40:], {c: round(x/1e6,3) for c,x in v.items()})
"
