# A/B of library builds on the lego bench (GPU box):
#   bash tools/ab_libs.sh name1 name2 ...   (name "base" = libgsmpm.so, else libgsmpm_<name>.so)
# extra bench args via BENCH_ARGS
set -e
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else L=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$v.so; fi
    GSMPM_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 $BENCH_ARGS > gpurun_out/ab_${v}_${rep}.json 2> gpurun_out/ab_${v}_${rep}.err
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${v}_${rep}.json')); print('$v', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], d.get('kernels_ms_per_launch_steady'))"
  done
done
