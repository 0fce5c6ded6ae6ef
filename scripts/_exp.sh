set -u
mkdir -p gpurun_out
for polls in 3 4 6; do
  RP_DEFER_POLLS=$polls timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kp.json 2> gpurun_out/kp.err || { tail -5 gpurun_out/kp.err; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/kp.json'));print('kdd polls=$polls', round(d['roofline']['kernel_ms'],2), d['deferred_tiles'])"
  RP_DEFER_POLLS=$polls timeout -k 10 400 python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4p.json 2> gpurun_out/c4p.err || { tail -5 gpurun_out/c4p.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4p.json'));print('cfg4 polls=$polls', round(d['roofline']['kernel_ms'],2), d['deferred_tiles'])"
done
