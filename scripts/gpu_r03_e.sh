#!/bin/bash
# round-3 session E: configs[3] full-size test, boundary-2/3 bench lines, configs[3] wave-state PMC,
# dense MFMA utilisation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -s -x -k configs3_full --timeout 500 --timeout-method thread > gpurun_out/r03e_cfg3.log 2>&1
rc=$?
grep -E "PASSED|FAILED|before configs|A ready" gpurun_out/r03e_cfg3.log | tail -4
[ $rc -ne 0 ] && { grep -n "Error" gpurun_out/r03e_cfg3.log | head -5; exit $rc; }
timeout -k 10 300 python -u bench.py --boundary host --steps 3 --warmup 1 > gpurun_out/r03_bench_host.json 2> gpurun_out/r03_bench_host.err || { tail -20 gpurun_out/r03_bench_host.err; exit 4; }
cut -c1-300 gpurun_out/r03_bench_host.json
timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 > gpurun_out/r03_bench_libsvm.json 2> gpurun_out/r03_bench_libsvm.err || { tail -20 gpurun_out/r03_bench_libsvm.err; exit 5; }
cut -c1-400 gpurun_out/r03_bench_libsvm.json
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -T --output-format csv -d gpurun_out/cfg4_wave -o pmc -- python3 bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/cfg4_wave.log 2>&1 || { tail -20 gpurun_out/cfg4_wave.log; exit 6; }
python3 scripts/pmc_kernels.py gpurun_out/cfg4_wave > gpurun_out/cfg4_wave.json && head -c 1500 gpurun_out/cfg4_wave.json
bash scripts/gpu_dense_pmc.sh > gpurun_out/dense_pmc.log 2>&1 || { tail -20 gpurun_out/dense_pmc.log; exit 7; }
for c in bf16 fp32; do python3 -c "import json;d=json.load(open('gpurun_out/dense_pmc_$c.json'));print('$c', {k: {c2: round(v2, 4) for c2, v2 in v.items() if 'Util' in c2 or 'Flops' in c2} for k, v in d.items()})"; done
