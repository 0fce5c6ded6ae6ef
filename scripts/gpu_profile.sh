#!/bin/bash
# Profiling session: full-size bench (configs[1]) + rocprofv3 kernel trace/stats + separate PMC passes,
# summarised into profiles/<TAG>_* (scripts/summarize_profile.py). Every GPU step has its own time
# limit; the first failure ends the session.
#   TAG=r02 BENCH_ARGS="..." PROF_ARGS="..." bash scripts/gpu_profile.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${TAG:-r02}"
BA="${BENCH_ARGS:---steps 10 --warmup 3}"
PA="${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline}"
run() { echo "== $*" >&2; "$@"; }
if [ -z "${SKIP_BENCH:-}" ]; then
  run timeout -k 10 600 python -u bench.py $BA > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 4; }
  cat gpurun_out/${TAG}_bench.json
fi
run timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_trace -o trace -- python3 bench.py $PA > gpurun_out/prof_${TAG}_bench.json 2> gpurun_out/prof_${TAG}_trace.log || { tail -20 gpurun_out/prof_${TAG}_trace.log; exit 5; }
PMCS="${PMCS:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"
IFS=';' read -ra GS <<< "$PMCS"
for pmc in "${GS[@]}"; do
  name=$(echo $pmc | tr ' ' '_')
  run timeout -s KILL 300 rocprofv3 --pmc $pmc -T --output-format csv -d gpurun_out/prof_${TAG}_pmc_$name -o pmc -- python3 bench.py $PA > gpurun_out/prof_${TAG}_pmc_$name.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_pmc_$name.log; exit 6; }
done
PROBE=""
if [ -n "${PROBE_LIB:-}" ]; then  # the gather probe build: one L2 pass (the W32 lookups' own hit rate)
  run timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/prof_${TAG}_probe -o pmc -- python3 bench.py $PA --lib $PROBE_LIB > gpurun_out/prof_${TAG}_probe.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_probe.log; exit 7; }
  PROBE="--probe-pmc gpurun_out/prof_${TAG}_probe"
fi
python3 scripts/summarize_profile.py --tag $TAG ${SUM_ARGS:-} $PROBE --bench-json gpurun_out/prof_${TAG}_bench.json > gpurun_out/summary_$TAG.json && tail -30 gpurun_out/summary_$TAG.json
exit 0
