# A/B of an env toggle on the lego bench (GPU box): bash tools/ab.sh VAR "a b" [extra bench args]
set -e
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  for rep in 1 2; do
    env $VAR=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 "$@" > gpurun_out/ab_${v}_${rep}.json 2> gpurun_out/ab_${v}_${rep}.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${v}_${rep}.json')); print('$VAR=$v', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], d['roofline']['frac'])"
  done
done
