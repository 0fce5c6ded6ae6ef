set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/g16.so abvar/m1g16.so abvar/m1g8.so" bash scripts/gpu_kstats.sh > gpurun_out/r06d_kstats.txt 2>&1; grep "==\|gather\|partition\|wave" gpurun_out/r06d_kstats.txt
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r06d_counters.txt 2>&1 || true
BA="--steps 1 --warmup 0 --no-cpu-baseline --host-steps 0"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc -T --output-format csv -d gpurun_out/r06d_sq_$i -o pmc -- python3 bench.py $BA > gpurun_out/r06d_sq_$i.log 2>&1 || { tail -20 gpurun_out/r06d_sq_$i.log; exit 6; }
done
python3 scripts/pmc_kernels.py gpurun_out/r06d_sq > gpurun_out/r06d_sq_kernels.json && python3 -c "
import json; d=json.load(open('gpurun_out/r06d_sq_kernels.json'))
for k,v in d.items():
    if 'lpr_' in k: print(k[-40:], {c: round(x/1e6,2) for c,x in v.items()})
"
