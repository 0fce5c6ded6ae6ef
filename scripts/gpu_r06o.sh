set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for sh in 19 18 20 19 18; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-steps 0 --stage-shift $sh > gpurun_out/r06o_b.json 2>gpurun_out/r06o_b.err || { tail -5 gpurun_out/r06o_b.err; exit 7; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r06o_b.json').read().strip().splitlines()[-1]); print('shift $sh', round(d['ms_per_step'],3), d['verified']['sample_bitexact_vs_oracle'])"
done
BENCH="--stage-shift 18" bash scripts/gpu_kstats.sh > gpurun_out/r06o_kstats.txt 2>&1; grep "==\|wave\|gather\|partition\|copy" gpurun_out/r06o_kstats.txt
