set -u
mkdir -p gpurun_out
for rep in 1 2; do
for sig in 1 0; do
  if [ $sig = 0 ]; then export RP_NO_SIGNATURES=1; else unset RP_NO_SIGNATURES; fi
  timeout -k 10 400 python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/sig_c4.json 2> gpurun_out/sig_c4.err || { tail -5 gpurun_out/sig_c4.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/sig_c4.json'));print('cfg4 sig=$sig', round(d['roofline']['kernel_ms'],2), d['deferred_tiles'])"
done
done
