set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/gw12.so" bash scripts/gpu_kstats.sh > gpurun_out/r06r_kstats_sb19.txt 2>&1 || { cat gpurun_out/r06r_kstats_sb19.txt; exit 6; }
cat gpurun_out/r06r_kstats_sb19.txt | grep "==\|gather\|wave\|partition"
BENCH="--staging on --stage-shift 18" LIBS="abvar/gw12.so" bash scripts/gpu_kstats.sh > gpurun_out/r06r_kstats_sb18.txt 2>&1 || { cat gpurun_out/r06r_kstats_sb18.txt; exit 7; }
cat gpurun_out/r06r_kstats_sb18.txt | grep "==\|gather\|wave\|partition\|copy"
