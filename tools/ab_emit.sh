# A/B of the emission kernels on one box: tools/render_probe.py (the render
# alone) with the balanced k_emit_wg (default) and the per-lane k_emit_pairs
# (GSMPM_RASTER_EMIT_LANE=1), bicycle (1M / 256^3) and lego, 3 interleaved
# pairs, then a rocprofv3 kernel-stats pass of each on the bicycle.
set -e
O=${1:-gpurun_out/ab_emit}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for l in 0 1; do
    GSMPM_RASTER_EMIT_LANE=$l CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 python3 tools/render_probe.py > $O/bicycle.l$l.$i.log 2>&1
    echo "bicycle emit_lane=$l $(tail -n 1 $O/bicycle.l$l.$i.log)"
    GSMPM_RASTER_EMIT_LANE=$l timeout -k 10 120 python3 tools/render_probe.py > $O/lego.l$l.$i.log 2>&1
    echo "lego emit_lane=$l $(tail -n 1 $O/lego.l$l.$i.log)"
  done
done
for l in 0 1; do
  GSMPM_RASTER_EMIT_LANE=$l CONFIG=bicycle.json N=1000000 NG=256 REPS=5 timeout -k 10 240 \
    rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$l -o run -- python3 tools/render_probe.py > $O/prof$l.log 2>&1
  f=$(find $O/prof$l -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/bicycle_kernel_stats_l$l.csv
done
echo ok
