#!/bin/bash
# Secondary measurements: configs[3] (power-law 100 nnz/row), configs[4] dense (fp32, bf16), and the
# host boundary (PCIe-inclusive, drop-in partition function). Each step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u bench.py --config cfg4 --steps 3 --warmup 1 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail -20 gpurun_out/bench_cfg4.err; exit 4; }
cat gpurun_out/bench_cfg4.json
for c in fp32 bf16; do
  timeout -k 10 300 python3 -u scripts/bench_dense.py --compute $c > gpurun_out/bench_dense_$c.json 2> gpurun_out/bench_dense_$c.err || { tail -20 gpurun_out/bench_dense_$c.err; exit 5; }
  cat gpurun_out/bench_dense_$c.json
done
timeout -k 10 400 python3 -u scripts/bench_host.py > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err || { tail -20 gpurun_out/bench_host.err; exit 6; }
cat gpurun_out/bench_host.json
