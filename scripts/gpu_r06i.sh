set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/head.so abvar/w8.so" ROUNDS=3 bash scripts/gpu_ab.sh
