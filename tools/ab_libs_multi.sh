# Interleaved A/B of library variants (GSMPM_LIB) on several configs.
# Usage: VARIANTS="base ps16 ps18" CONFIGS="B C Bp" REPS=2 bash tools/ab_libs_multi.sh <outdir>
# variant "base" = libgsmpm.so, any other name = libgsmpm_<name>.so
set -o pipefail
O=${1:-gpurun_out/ab_libs}; mkdir -p $O
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/$lib timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs "$@" > $O/${name}.json 2> $O/${name}.err || { tail -5 $O/${name}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${name}.json')); print('$name', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], 'esc', d.get('escapes_timed'))"
}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    lib=libgsmpm.so; [ $v != base ] && lib=libgsmpm_$v.so
    for c in ${CONFIGS:-B}; do
      case $c in
        B) run B_${v}_${rep} $lib --steps 20 --warmup 3 || exit 1;;
        C) run C_${v}_${rep} $lib --steps 20 --warmup 3 --config lego-fracture.json --material metal || exit 1;;
        Bp) run Bp_${v}_${rep} $lib --steps 10 --warmup 3 --particles 240549 || exit 1;;
        D) run D_${v}_${rep} $lib --steps 4 --warmup 2 --config bicycle.json --particles 1000000 --n_grid 256 || exit 1;;
      esac
    done
  done
done
