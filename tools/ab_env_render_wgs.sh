# A/B: k_render's grid (GSMPM_RASTER_RENDER_WGS) on the default lego bench frame
set -e
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for W in 0 64 128 256 512; do
    GSMPM_RASTER_RENDER_WGS=$W timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > gpurun_out/ab/wgs_${W}_${rep}.json 2> gpurun_out/ab/wgs_${W}_${rep}.err
    python3 -c "import json; d=json.load(open('gpurun_out/ab/wgs_${W}_${rep}.json')); print('wgs $W', round(d['value']/1e9,4), 'frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', d.get('render_ms_per_frame'))"
  done
done
