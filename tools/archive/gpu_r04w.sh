# Round 4, GPU call W: with the render now overlapping the simulator (render
# worker thread), a k_render of fewer workgroups looping over quarters
# (GSMPM_RASTER_RENDER_WGS) might take fewer CU slots at once: lego bench, 3
# interleaved rounds.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
for i in 1 2 3; do for w in 0 64 128 256; do
  if [ $w -eq 0 ]; then unset GSMPM_RASTER_RENDER_WGS; else export GSMPM_RASTER_RENDER_WGS=$w; fi
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > $O/w_${w}_$i.json 2> $O/w_${w}_$i.err || { tail -5 $O/w_${w}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/w_${w}_$i.json')); print('render_wgs=$w', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', round(d['render_ms_per_frame'],4))"
done; done | tee $O/ab_render_wgs.txt
