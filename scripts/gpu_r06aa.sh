set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/w6.so abvar/w8.so" bash scripts/gpu_kstats.sh > gpurun_out/r06aa_kstats.txt 2>&1 || { cat gpurun_out/r06aa_kstats.txt; exit 6; }
grep "==\|wave" gpurun_out/r06aa_kstats.txt
for f in 1 2 3; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/ks_$f.json').read().strip().splitlines()[-1]); print($f, d['ms_per_step'])"; done
LIBS="abvar/sc23.so" BENCH="--config cfg4 --steps 3 --warmup 1" bash scripts/gpu_kstats.sh > gpurun_out/r06aa_kstats4.txt 2>&1 || { cat gpurun_out/r06aa_kstats4.txt; exit 7; }
cat gpurun_out/r06aa_kstats4.txt
