# A/B of a raster environment switch on one build (render alone,
# tools/render_probe.py): bicycle and lego, 3 interleaved rounds.
#   bash tools/ab_env_render.sh VAR "VALUE_A VALUE_B ..." [out]
set -e
V=$1; VALS=$2; O=${3:-gpurun_out/ab_env_render}
mkdir -p $O
for i in 1 2 3; do
  for L in $VALS; do
    env $V=$L CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 python3 tools/render_probe.py > $O/bicycle.$L.$i.log 2>&1
    echo "bicycle $V=$L $(tail -n 1 $O/bicycle.$L.$i.log)"
    env $V=$L REPS=50 timeout -k 10 120 python3 tools/render_probe.py > $O/lego.$L.$i.log 2>&1
    echo "lego $V=$L $(tail -n 1 $O/lego.$L.$i.log)"
  done
done
