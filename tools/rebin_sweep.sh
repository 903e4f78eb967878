# The re-binning-interval pathology (round-5 verdict item 3): the lego bench
# at several intervals R, each line with its escapes (particle scatters that
# left their chunk window -> an all-tile k_grid_f sweep) in the timed frames,
# the timed frame and the sim-only frame.  GPU box.  Usage: bash tools/rebin_sweep.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/rebin}; mkdir -p $O
for rep in $(seq 1 ${REPS:-1}); do
  for R in ${RS:-10 20 25 30 40 50}; do
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 5 --rebin $R $BENCH_ARGS > $O/R${R}_${rep}.json 2> $O/R${R}_${rep}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/R${R}_${rep}.json')); print('R', $R, 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'esc_timed', d['escapes_timed'], 'esc_total', d['escapes_since_start'], d['kernels_ms_per_launch'])"
  done
done
