# A/B of the metal stress-path builds on lego-fracture --material metal (GPU box):
# base = libgsmpm.so, others libgsmpm_<name>.so; REPS interleaved rounds.
set -o pipefail
O=${1:-gpurun_out/ab_metal}; shift; mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else L=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$v.so; fi
    GSMPM_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 5 --config lego-fracture.json --material metal > $O/${v}_${rep}.json 2> $O/${v}_${rep}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/${v}_${rep}.json')); print('$v', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'])"
  done
done
