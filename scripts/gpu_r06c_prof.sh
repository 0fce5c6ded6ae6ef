set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06c SKIP_BENCH=1 PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --host-steps 0" bash scripts/gpu_profile.sh > gpurun_out/r06c_prof.log 2>&1 || { tail -5 gpurun_out/r06c_prof.log; exit 4; }
tail -3 gpurun_out/r06c_prof.log
TAG=r06c_cfg4 SKIP_BENCH=1 PMCS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" PROF_ARGS="--config cfg4 --steps 2 --warmup 1 --no-cpu-baseline" SUM_ARGS="--rows 200000000 --dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r06c_cfg4_prof.log 2>&1; rc=$?
tail -3 gpurun_out/r06c_cfg4_prof.log
exit $rc
