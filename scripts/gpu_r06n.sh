set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/bloomall.so" ROUNDS=3 bash scripts/gpu_ab.sh
LIBS="abvar/bloomall.so" bash scripts/gpu_kstats.sh > gpurun_out/r06n_kstats.txt 2>&1; grep "==\|wave" gpurun_out/r06n_kstats.txt
