#!/bin/bash
# Round-3 bench lines + profiles on the final sources. PART=1: configs[1] default line (with the CPU
# reference) + kernel stats + PMC passes (profiles/r03_*); PART=2: power-law columns and configs[3];
# PART=3: boundary-2/3 lines and the dense MFMA utilisation. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PM="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
case "${PART:-1}" in
1)
  timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -20 gpurun_out/r03_bench.err; exit 4; }
  cut -c1-400 gpurun_out/r03_bench.json
  PMCS="$PM" SKIP_BENCH=1 TAG=r03 bash scripts/gpu_profile.sh > gpurun_out/r03_prof.log 2>&1 || { tail -20 gpurun_out/r03_prof.log; exit 5; }
  ;;
2)
  PMCS="$PM" SKIP_BENCH=1 TAG=r03_powerlaw PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --dist powerlaw" \
    SUM_ARGS="--dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r03_powerlaw_prof.log 2>&1 || { tail -20 gpurun_out/r03_powerlaw_prof.log; exit 5; }
  timeout -k 10 900 python -u bench.py --config cfg4 --steps 3 --warmup 1 > gpurun_out/r03_bench_cfg4.json 2> gpurun_out/r03_bench_cfg4.err || { tail -20 gpurun_out/r03_bench_cfg4.err; exit 6; }
  cut -c1-400 gpurun_out/r03_bench_cfg4.json
  PMCS="$PM" SKIP_BENCH=1 TAG=r03_cfg4 PROF_ARGS="--config cfg4 --steps 2 --warmup 1 --no-cpu-baseline" \
    SUM_ARGS="--rows 200000000 --dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r03_cfg4_prof.log 2>&1 || { tail -20 gpurun_out/r03_cfg4_prof.log; exit 7; }
  ;;
3)
  timeout -k 10 300 python -u bench.py --boundary host --steps 3 --warmup 1 > gpurun_out/r03_bench_host.json 2> gpurun_out/r03_bench_host.err || { tail -20 gpurun_out/r03_bench_host.err; exit 4; }
  cut -c1-300 gpurun_out/r03_bench_host.json
  timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 > gpurun_out/r03_bench_libsvm.json 2> gpurun_out/r03_bench_libsvm.err || { tail -20 gpurun_out/r03_bench_libsvm.err; exit 5; }
  cut -c1-400 gpurun_out/r03_bench_libsvm.json
  bash scripts/gpu_dense_pmc.sh > gpurun_out/dense_pmc.log 2>&1 || { tail -20 gpurun_out/dense_pmc.log; exit 7; }
  for c in bf16 fp32; do python3 -c "import json;d=json.load(open('gpurun_out/dense_pmc_$c.json'));print('$c', {k: {c2: round(v2, 4) for c2, v2 in v.items()} for k, v in d.items() if 'dense' in k})"; done
  ;;
esac
echo done
