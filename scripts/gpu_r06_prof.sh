set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06 SKIP_BENCH=1 PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --host-steps 0" PROBE_LIB=abvar/gather_now32.so bash scripts/gpu_profile.sh > gpurun_out/r06_prof.log 2>&1; rc=$?
tail -5 gpurun_out/r06_prof.log
[ $rc -eq 0 ] || exit $rc
LIBS="abvar/gather_now32.so" bash scripts/gpu_kstats.sh > gpurun_out/r06_probe_kstats.txt 2>&1; grep "==\|gather" gpurun_out/r06_probe_kstats.txt
