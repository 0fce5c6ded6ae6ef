set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err || { tail -5 gpurun_out/r06b_bench.err; exit 4; }
tail -c 300 gpurun_out/r06b_bench.json; echo
timeout -k 10 400 python -u bench.py --dist powerlaw --steps 20 --warmup 5 --host-steps 3 --no-cpu-baseline > gpurun_out/r06b_bench_powerlaw.json 2> gpurun_out/r06b_bench_powerlaw.err || { tail -5 gpurun_out/r06b_bench_powerlaw.err; exit 5; }
timeout -k 10 400 python -u bench.py --config kdd9x --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06b_bench_kdd9x.json 2> gpurun_out/r06b_bench_kdd9x.err || { tail -5 gpurun_out/r06b_bench_kdd9x.err; exit 6; }
timeout -k 10 400 python -u bench.py --boundary libsvm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06b_bench_libsvm.json 2> gpurun_out/r06b_bench_libsvm.err || { tail -5 gpurun_out/r06b_bench_libsvm.err; exit 7; }
echo bench-done
TAG=r06b_cfg4 SKIP_BENCH=1 PMCS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" PROF_ARGS="--config cfg4 --steps 2 --warmup 1 --no-cpu-baseline" SUM_ARGS="--rows 200000000 --dist powerlaw --no-latest" bash scripts/gpu_profile.sh > gpurun_out/r06b_cfg4_prof.log 2>&1; rc=$?
tail -3 gpurun_out/r06b_cfg4_prof.log
exit $rc
