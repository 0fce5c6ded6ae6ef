set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config cfg4 --steps 5 --warmup 2 > gpurun_out/r06_bench_cfg4.json 2> gpurun_out/r06_bench_cfg4.err || { tail -5 gpurun_out/r06_bench_cfg4.err; exit 4; }
tail -c 300 gpurun_out/r06_bench_cfg4.json
