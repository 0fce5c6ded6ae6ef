#!/bin/bash
# round-3: where boundary 3's time goes — kernel trace of bench.py --boundary libsvm, and the line at
# two chunk sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/lsv_trace -o t -- python3 bench.py --boundary libsvm --steps 2 --warmup 1 > gpurun_out/lsv_trace.log 2>&1 || { tail -20 gpurun_out/lsv_trace.log; exit 4; }
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/lsv_trace/**/t_kernel_stats.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)/1e6
print('kernels total ms (3 calls):', round(tot,1))
for r in rows[:12]: print(r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms')"
for cb in 33554432 134217728; do
  timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 --chunk-bytes $cb > gpurun_out/lsv_$cb.json 2> gpurun_out/lsv_$cb.err || { tail -20 gpurun_out/lsv_$cb.err; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/lsv_$cb.json'));print('chunk $cb', round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],1), 'ms')"
done
