set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06b SKIP_BENCH=1 PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --host-steps 0" bash scripts/gpu_profile.sh > gpurun_out/r06b_prof.log 2>&1; rc=$?
tail -5 gpurun_out/r06b_prof.log
exit $rc
