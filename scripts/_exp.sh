set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/pytest_defer.log 2>&1 || { tail -30 gpurun_out/pytest_defer.log; exit 3; }
tail -2 gpurun_out/pytest_defer.log
for polls in -1 0 2 8; do
  for mode in off on; do
    RP_DEFER_POLLS=$polls timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --staging $mode > gpurun_out/defer_${polls}_$mode.json 2>gpurun_out/defer_${polls}_$mode.err || { tail -5 gpurun_out/defer_${polls}_$mode.err; exit 5; }
    python3 -c "import json;d=json.load(open('gpurun_out/defer_${polls}_$mode.json'));print('polls=$polls mode=$mode', round(d['roofline']['kernel_ms'],2))"
  done
done
