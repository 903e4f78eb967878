# A/B of the escape handling on the GPU box: the touched-tile form (default:
# escaped particles add their stencil tiles to the touched list) against
# round 5's all-tile sweep (libgsmpm_escsweep.so, -DGSMPM_ESC_SWEEP=1), on the
# lego bench at the default re-binning interval (B), at 50 substeps (B50, the
# interval that escaped most), B' and metal (C, no escapes).
# Usage: bash tools/ab_esc.sh <outdir>; REPS interleaved rounds.
set -o pipefail
O=${1:-gpurun_out/ab_esc}; mkdir -p $O
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/$lib timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs "$@" > $O/${name}.json 2> $O/${name}.err || { tail -5 $O/${name}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${name}.json')); print('$name', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'], 'esc', d.get('escapes_timed'))"
}
for rep in $(seq 1 ${REPS:-2}); do
  for v in sweep touched; do
    lib=libgsmpm.so; [ $v = sweep ] && lib=libgsmpm_escsweep.so
    case " ${CONFIGS:-B B50 Bp C} " in *" B "*) run B_${v}_${rep} $lib --steps 20 --warmup 3 || exit 1;; esac
    case " ${CONFIGS:-B B50 Bp C} " in *" B50 "*) run B50_${v}_${rep} $lib --steps 20 --warmup 3 --rebin 50 || exit 1;; esac
    case " ${CONFIGS:-B B50 Bp C} " in *" Bp "*) run Bp_${v}_${rep} $lib --steps 10 --warmup 3 --particles 240549 || exit 1;; esac
    case " ${CONFIGS:-B B50 Bp C} " in *" C "*) run C_${v}_${rep} $lib --steps 20 --warmup 3 --config lego-fracture.json --material metal || exit 1;; esac
  done
done
