#!/bin/bash
# Separate rocprofv3 --pmc passes over a short bench.py run (one pass per counter group, each under
# its own kill timeout), summarised per kernel. Usage: TAG=name BENCH="--staging on" bash scripts/gpu_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${TAG:-pmc}"
BA="--steps 1 --warmup 0 --no-cpu-baseline ${BENCH:-}"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc -T --output-format csv -d gpurun_out/${TAG}_$i -o pmc -- python3 bench.py $BA > gpurun_out/${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_$i.log; exit 6; }
done
python3 scripts/pmc_kernels.py gpurun_out/${TAG} > gpurun_out/${TAG}_kernels.json && cat gpurun_out/${TAG}_kernels.json
