# A/B of the size-balanced chunk order (k_chunk_order, GSMPM_CHUNK_ORDER) on
# the lego bench (B), lego-fracture metal (C), B' (240,549) and bicycle (D,
# fewer frames), REPS interleaved rounds.  Usage: bash tools/ab_order.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/ab_order}; mkdir -p $O
run() {  # name order args...
  local name=$1 ord=$2; shift 2
  GSMPM_CHUNK_ORDER=$ord timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs "$@" > $O/${name}.json 2> $O/${name}.err || { tail -5 $O/${name}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${name}.json')); print('$name', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], 'esc', d.get('escapes_timed'))"
}
for rep in $(seq 1 ${REPS:-2}); do
  for ord in 0 1; do
    run B_o${ord}_${rep} $ord --steps 20 --warmup 3 || exit 1
    run C_o${ord}_${rep} $ord --steps 20 --warmup 3 --config lego-fracture.json --material metal || exit 1
    run Bp_o${ord}_${rep} $ord --steps 10 --warmup 3 --particles 240549 || exit 1
    run D_o${ord}_${rep} $ord --steps 4 --warmup 2 --config bicycle.json --particles 1000000 --n_grid 256 || exit 1
  done
done
