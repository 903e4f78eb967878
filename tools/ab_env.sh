# A/B of an env setting on the lego bench (GPU box): bash tools/ab_env.sh "VAR=a" "VAR=b" ...
set -e
for rep in 1 2; do
  for kv in "$@"; do
    env $kv timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 $BENCH_ARGS > gpurun_out/abe_${rep}.json 2> gpurun_out/abe_${rep}.err
    python3 -c "import json; d=json.load(open('gpurun_out/abe_${rep}.json')); print('$kv', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], d.get('kernels_ms_per_launch_steady'))"
  done
done
