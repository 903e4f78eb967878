# A/B of the adaptive re-binning count (round 6) on the lego bench and on
# lego-fracture --material metal: fixed spacing (GSMPM_REBIN_AUTO=0, the
# material default 20) against the adaptive count with the default longest
# spacing and with longer ones (libgsmpm_sf50 / st25 / st50: GSMPM_REBIN_SF /
# GSMPM_REBIN_STRESS).  REPS interleaved rounds.  GPU box.
set -o pipefail
O=${1:-gpurun_out/ab_rebin}; mkdir -p $O
G=$PWD/gaussian-splatting-mpm_amd
one() {  # one <name> <lib> <auto> <bench args...>
  local n=$1 L=$2 A=$3; shift 3
  GSMPM_REBIN_AUTO=$A GSMPM_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || return 1
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'esc_timed', d['escapes_timed'], d['rebin'])"
}
for rep in $(seq 1 ${REPS:-2}); do
  one lego_fixed20_$rep $G/libgsmpm.so 0 || exit 1
  one lego_auto20_$rep $G/libgsmpm.so 1 || exit 1
  one lego_auto50_$rep $G/libgsmpm_sf50.so 1 || exit 1
  one metal_fixed20_$rep $G/libgsmpm.so 0 --material metal || exit 1
  one metal_auto20_$rep $G/libgsmpm.so 1 --material metal || exit 1
  one metal_auto25_$rep $G/libgsmpm_st25.so 1 --material metal || exit 1
  one metal_auto50_$rep $G/libgsmpm_st50.so 1 --material metal || exit 1
done
