#!/bin/bash
# boundary 3 timeline: kernel + memory-copy trace of the libsvm bench (csv under gpurun_out/tr_libsvm)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr_libsvm -o run -- python3 bench.py --boundary libsvm --steps 2 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/tr_libsvm.json 2> gpurun_out/tr_libsvm.err || { tail -20 gpurun_out/tr_libsvm.err; exit 5; }
python3 scripts/timeline_summary.py gpurun_out/tr_libsvm
