#!/bin/bash
# rocprofv3 --pmc passes (one group per run, own kill timeout) over a 1-step bench.py; per-kernel
# means. Usage: TAG=name BENCH="..." GROUPS_="g1;g2" bash scripts/gpu_pmc2.sh  (env as exported)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${TAG:-pmc}"
BA="--steps 1 --warmup 0 --no-cpu-baseline ${BENCH:-}"
IFS=';' read -ra GS <<< "${GROUPS_:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum}"
i=0
for pmc in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc -T --output-format csv -d gpurun_out/${TAG}_$i -o pmc -- python3 bench.py $BA > gpurun_out/${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_$i.log; exit 6; }
done
python3 scripts/pmc_kernels.py gpurun_out/${TAG} > gpurun_out/${TAG}_kernels.json
python3 - gpurun_out/${TAG}_kernels.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if any(s in k for s in ("lpr_", "stage_", "spgemm", "defer_copy")):
        print(k[:40], {c: (f"{x:.4g}") for c, x in v.items()})
PY
