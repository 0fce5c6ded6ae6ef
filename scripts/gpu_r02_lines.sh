#!/bin/bash
# Round-2 bench lines + profiles. PART=1: configs[1] default line (with the CPU reference) and its
# rocprofv3 kernel stats + PMC passes (profiles/r02_*); PART=2: power-law columns and configs[3]
# (200M x 10M, 100 nnz/row), each with kernel stats and PMC passes. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PM="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { tail -20 gpurun_out/r02_bench.err; exit 4; }
  cat gpurun_out/r02_bench.json
  PMCS="$PM" SKIP_BENCH=1 TAG=r02 bash scripts/gpu_profile.sh > gpurun_out/r02_prof.log 2>&1 || { tail -20 gpurun_out/r02_prof.log; exit 5; }
else
  PMCS="$PM" SKIP_BENCH=1 TAG=r02_powerlaw PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --dist powerlaw" \
    SUM_ARGS="--dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r02_powerlaw_prof.log 2>&1 || { tail -20 gpurun_out/r02_powerlaw_prof.log; exit 5; }
  timeout -k 10 900 python -u bench.py --config cfg4 --steps 3 --warmup 1 > gpurun_out/r02_bench_cfg4.json 2> gpurun_out/r02_bench_cfg4.err || { tail -20 gpurun_out/r02_bench_cfg4.err; exit 6; }
  cat gpurun_out/r02_bench_cfg4.json
  PMCS="$PM" SKIP_BENCH=1 TAG=r02_cfg4 PROF_ARGS="--config cfg4 --steps 2 --warmup 1 --no-cpu-baseline" \
    SUM_ARGS="--rows 200000000 --dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r02_cfg4_prof.log 2>&1 || { tail -20 gpurun_out/r02_cfg4_prof.log; exit 7; }
fi
echo done
