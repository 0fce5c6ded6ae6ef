#!/bin/bash
# round-3 session J: per-kernel times of two librp builds on configs[1] (rocprofv3 kernel trace),
# then in-kernel stage stamps of the current sources (librp_diag.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for lib in ${LIBS:-randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so}; do
  i=$((i + 1))
  RP_LIB=$lib timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/j_prof_$i -o t -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/j_prof_$i.log 2>&1 || { tail -20 gpurun_out/j_prof_$i.log; exit 4; }
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/j_prof_$i/**/t_kernel_stats.csv',recursive=True)[0]
rows=[r for r in csv.DictReader(open(f)) if r['Name'].startswith(('lpr_','spgemm_','stage_','defer_'))]
print('$lib', ' '.join('%s=%.3f'%(r['Name'],float(r['AverageNs'])/1e6) for r in rows))"
done
timeout -k 10 300 python -u scripts/stage_stamps.py --rows 119705032 --p 4096 --lpr --staging on > gpurun_out/j_stamps.log 2>&1 || { tail -5 gpurun_out/j_stamps.log; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/stamps.json'));print({k:(v if not isinstance(v,dict) else {a:round(b,2) for a,b in v.items()}) for k,v in d.items()})"
