#!/bin/bash
# round-4 bench lines on the final sources: power-law columns, configs[2] (kdd9x) and configs[3]
# (cfg4) on one GPU, boundaries 2 (host CSR), 3 (libsvm) and the drop-in partition function
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > gpurun_out/r04_bench_$name.json 2> gpurun_out/r04_bench_$name.err || { tail -20 gpurun_out/r04_bench_$name.err; exit 4; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04_bench_$name.json'));print('$name', round(d['value']/1e6,2), 'M', d['unit'], round(d['ms_per_step'],2), 'ms', (d.get('roofline') or {}).get('frac'))"
}
line powerlaw 400 --dist powerlaw --steps 10 --warmup 3 --no-cpu-baseline
line kdd9x 500 --config kdd9x --steps 3 --warmup 1 --no-cpu-baseline
line cfg4 600 --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline
line host 400 --boundary host --steps 5 --warmup 2 --no-cpu-baseline
line libsvm 400 --boundary libsvm --steps 5 --warmup 2 --no-cpu-baseline
line partition 500 --boundary partition --steps 2 --warmup 1
