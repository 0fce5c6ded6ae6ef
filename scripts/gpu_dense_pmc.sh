#!/bin/bash
# configs[4] dense path: MFMA utilisation and MFMA FLOPs by input type from rocprofv3's derived
# counters (MfmaUtil = sum SQ_VALU_MFMA_BUSY_CYCLES / (max GRBM_GUI_ACTIVE x SIMDs); MfmaFlops* =
# SQ_INSTS_VALU_MFMA_MOPS_* x 512), one pass each, fp32 and bf16; plus the kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${COMPUTES:-bf16 fp32 fp64}; do
  i=0
  for pmc in "MfmaUtil" "MfmaFlopsBF16 MfmaFlopsF32 MfmaFlopsF64"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pmc -T --output-format csv -d gpurun_out/dense_pmc_${c}_$i -o pmc -- python3 scripts/bench_dense.py --compute $c --steps 3 --warmup 1 --no-stream > gpurun_out/dense_pmc_${c}_$i.log 2>&1 || { tail -20 gpurun_out/dense_pmc_${c}_$i.log; exit 6; }
  done
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/dense_trace_$c -o t -- python3 scripts/bench_dense.py --compute $c --steps 3 --warmup 1 --no-stream > gpurun_out/dense_trace_$c.log 2>&1 || { tail -20 gpurun_out/dense_trace_$c.log; exit 7; }
  python3 scripts/pmc_kernels.py gpurun_out/dense_pmc_${c}_ > gpurun_out/dense_pmc_$c.json
done
echo done
