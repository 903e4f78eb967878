# A/B of onesweep configs / the depth sort on the render alone (tools/render_probe.py), bicycle and lego,
# 3 interleaved rounds: base + variant libraries libgsmpm_<name>.so
set -e
O=gpurun_out/ab_os
mkdir -p $O
for i in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$v.so; fi
    GSMPM_LIB=$LIB CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 python3 tools/render_probe.py > $O/bicycle.$v.$i.log 2>&1
    echo "bicycle $v $(tail -n 1 $O/bicycle.$v.$i.log)"
    GSMPM_LIB=$LIB REPS=50 timeout -k 10 120 python3 tools/render_probe.py > $O/lego.$v.$i.log 2>&1
    echo "lego $v $(tail -n 1 $O/lego.$v.$i.log)"
  done
done
