#!/bin/bash
# round-3: dense GEMM ring depth A/B (variant 11: 4 stages, 12: 5 stages) + the dense tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dz_tests.log 2>&1
rc=$?
tail -2 gpurun_out/dz_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/dz_tests.log | head -8; exit $rc; }
for c in bf16 fp32; do for v in 11 12 11 12; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute $c --no-stream --variant $v > gpurun_out/dz_${c}_v$v.json 2> gpurun_out/dz_${c}_v$v.err || { tail -20 gpurun_out/dz_${c}_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/dz_${c}_v$v.json'));print('$c v$v', round(d['roofline']['achieved'],1), 'TF', d.get('rel_err_vs_fp64_same_operands',{}).get('librp'))"
done; done
# configs[1] wave states of the row-lane kernels (one PMC pass)
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -T --output-format csv -d gpurun_out/cfg1_wave -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg1_wave.log 2>&1 || { tail -20 gpurun_out/cfg1_wave.log; exit 7; }
python3 scripts/pmc_kernels.py gpurun_out/cfg1_wave > gpurun_out/cfg1_wave.json && python3 -c "
import json;d=json.load(open('gpurun_out/cfg1_wave.json'))
for k in ('lpr_main_kernel','lpr_gather_kernel','lpr_partition_kernel','lpr_copy_kernel'):
  v=d[k]; c=v['SQ_WAVE_CYCLES']; print(k, 'wait', round(v['SQ_WAIT_ANY']/c,3), 'inst_stall', round(v['SQ_WAIT_INST_ANY']/c,3), 'active', round(v['SQ_ACTIVE_INST_ANY']/c,3), 'valu', v['SQ_INSTS_VALU'])"
