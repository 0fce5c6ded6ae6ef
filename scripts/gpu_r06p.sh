set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 5; }
tail -3 gpurun_out/r06p_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "configs1" --timeout 500 --timeout-method thread > gpurun_out/r06p_full.log 2>&1 || { tail -30 gpurun_out/r06p_full.log; exit 6; }
tail -3 gpurun_out/r06p_full.log
LIBS="${LIBS:-abvar/head.so}" bash scripts/gpu_kstats.sh > gpurun_out/r06p_kstats.txt 2>&1; rc=$?
cat gpurun_out/r06p_kstats.txt
exit $rc
