#!/bin/bash
# round-3 session H: long-row wave pipeline grid fix; deferral budgets; wave-state counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_longrow.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_longrow.log 2>&1 || { tail -20 gpurun_out/r03h_longrow.log; exit 3; }
tail -1 gpurun_out/r03h_longrow.log
timeout -k 10 300 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --pipeline longrow > gpurun_out/h_cfg4.json 2> gpurun_out/h_cfg4.err || { tail -20 gpurun_out/h_cfg4.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/h_cfg4.json'));print('cfg4 longrow', round(d['ms_per_step'],3), 'ms', d['verified']['sample_bitexact_vs_oracle'], d['deferred_tiles'], d['tiles'])"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM -T --output-format csv -d gpurun_out/h_wave -o pmc -- python3 bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline --pipeline longrow > gpurun_out/h_wave.log 2>&1 || { tail -20 gpurun_out/h_wave.log; exit 6; }
python3 scripts/pmc_kernels.py gpurun_out/h_wave > gpurun_out/h_wave.json && python3 -c "import json;d=json.load(open('gpurun_out/h_wave.json'));[print(k, {c: '%.4g' % v for c, v in cs.items()}) for k, cs in d.items() if 'lrw' in k or 'lookback' in k]"
