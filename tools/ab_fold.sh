# A/B of the folded grid update on the lego bench (GPU box): GSMPM_FOLD=0 (a
# k_grid_f launch after every k_fused) against the fold with 1 (default) and
# 2 staged nodes in flight per lane.  REPS interleaved rounds.
set -o pipefail
O=${1:-gpurun_out/ab_fold}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for v in nofold base fb2; do
    L=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; F=1
    [ $v = nofold ] && F=0
    [ $v = fb2 ] && L=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$v.so
    GSMPM_FOLD=$F GSMPM_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 $BENCH_ARGS > $O/${v}_${rep}.json 2> $O/${v}_${rep}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/${v}_${rep}.json')); print('$v', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], 'esc', d.get('escapes_since_start'))"
  done
done
