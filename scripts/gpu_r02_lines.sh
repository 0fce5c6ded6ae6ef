#!/bin/bash
# Round-2 bench lines + profiles: configs[1] default line (with the CPU reference), the power-law
# column variant, and configs[3] (200M x 10M, 100 nnz/row), each with rocprofv3 kernel stats and
# PMC passes summarised into profiles/<tag>_*. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { tail -20 gpurun_out/r02_bench.err; exit 4; }
cat gpurun_out/r02_bench.json
PMCS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  SKIP_BENCH=1 TAG=r02_powerlaw PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --dist powerlaw" \
  SUM_ARGS="--dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r02_powerlaw_prof.log 2>&1 || { tail -20 gpurun_out/r02_powerlaw_prof.log; exit 5; }
timeout -k 10 900 python -u bench.py --config cfg4 --steps 3 --warmup 1 > gpurun_out/r02_bench_cfg4.json 2> gpurun_out/r02_bench_cfg4.err || { tail -20 gpurun_out/r02_bench_cfg4.err; exit 6; }
cat gpurun_out/r02_bench_cfg4.json
PMCS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  SKIP_BENCH=1 TAG=r02_cfg4 PROF_ARGS="--config cfg4 --steps 2 --warmup 1 --no-cpu-baseline" \
  SUM_ARGS="--rows 200000000 --dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r02_cfg4_prof.log 2>&1 || { tail -20 gpurun_out/r02_cfg4_prof.log; exit 7; }
echo done
