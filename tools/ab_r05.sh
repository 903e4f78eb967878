# Interleaved A/B of library builds and environment switches on the lego bench
# (GPU box).  usage: bash tools/ab_r05.sh OUT "name|lib|ENV=.. ENV2=.." ...
#   lib: "" = libgsmpm.so, else libgsmpm_<lib>.so; REPS rounds (default 3)
set -o pipefail
O=$1; shift
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    IFS='|' read -r name lib envs <<< "$spec"
    if [ -z "$lib" ]; then L=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else L=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$lib.so; fi
    env GSMPM_LIB=$L $envs timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 $BENCH_ARGS > $O/${name}_${rep}.json 2> $O/${name}_${rep}.err || { echo "FAIL $name"; tail -5 $O/${name}_${rep}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${name}_${rep}.json')); k=d['kernels_ms_per_launch']; print('$name', round(d['value']/1e9,4), 'frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'k_fused', round(k['k_fused']*1e3,2), 'k_grid_f', round(k['k_grid_f']*1e3,2), 'steady', {a: round(b*1e3,2) for a, b in d['kernels_ms_per_launch_steady'].items()})" | tee -a $O/summary.txt
  done
done
