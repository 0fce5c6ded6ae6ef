set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/t_nos2.so abvar/t_nolb.so abvar/t_none.so" BENCH="--config cfg4 --steps 3 --warmup 1" bash scripts/gpu_kstats.sh > gpurun_out/r06j_kstats.txt 2>&1; cat gpurun_out/r06j_kstats.txt
