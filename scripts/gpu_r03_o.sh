#!/bin/bash
# round-3 session O: per-kernel A/B of librp builds on configs[1] (no stamps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for lib in $LIBS; do
  i=$((i + 1))
  RP_LIB=$lib timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/o_prof_$i -o t -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/o_prof_$i.log 2>&1 || { tail -20 gpurun_out/o_prof_$i.log; exit 4; }
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/o_prof_$i/**/t_kernel_stats.csv',recursive=True)[0]
rows=[r for r in csv.DictReader(open(f)) if r['Name'].startswith(('lpr_','spgemm_','stage_','defer_'))]
print('$lib', 'sum=%.3f'%sum(float(r['AverageNs'])/1e6 for r in rows if r['Name']!='lpr_main_flat_kernel'), ' '.join('%s=%.3f'%(r['Name'],float(r['AverageNs'])/1e6) for r in rows))"
done
