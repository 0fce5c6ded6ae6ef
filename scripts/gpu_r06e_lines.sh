#!/bin/bash
# Round-6 final build: the power-law, configs[2] (kdd9x) and libsvm bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --dist powerlaw --steps 20 --warmup 5 --host-steps 3 --no-cpu-baseline > gpurun_out/r06e_bench_powerlaw.json 2> gpurun_out/r06e_bench_powerlaw.err || { tail -5 gpurun_out/r06e_bench_powerlaw.err; exit 5; }
timeout -k 10 400 python -u bench.py --config kdd9x --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06e_bench_kdd9x.json 2> gpurun_out/r06e_bench_kdd9x.err || { tail -5 gpurun_out/r06e_bench_kdd9x.err; exit 6; }
timeout -k 10 400 python -u bench.py --boundary libsvm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06e_bench_libsvm.json 2> gpurun_out/r06e_bench_libsvm.err || { tail -5 gpurun_out/r06e_bench_libsvm.err; exit 7; }
echo lines-done
