#!/bin/bash
# The gather probe (make_gather_probe.py) under rocprofv3: kernel stats + one L2 PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L="${LIB:-variants/gather_now32.so}"
PA="--steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --lib $L"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/probe_gather_trace -o trace -- python3 bench.py $PA > gpurun_out/probe_gather_bench.json 2> gpurun_out/probe_gather_trace.log || exit 5
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/probe_gather_pmc -o pmc -- python3 bench.py $PA > gpurun_out/probe_gather_pmc.log 2>&1 || exit 6
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -T --output-format csv -d gpurun_out/probe_gather_pmc2 -o pmc -- python3 bench.py $PA > gpurun_out/probe_gather_pmc2.log 2>&1 || exit 7
exit 0
