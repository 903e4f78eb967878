# A/B of the render kernels on one box: bench.py's render_ms_per_frame (the
# frame's render alone, 5 reps) with the per-quarter k_render (default) and
# k_render4 (GSMPM_RASTER_TILE_SHARED=1), 3 interleaved pairs.
set -e
O=${1:-gpurun_out/ab_render}
mkdir -p $O
for i in 1 2 3; do
  for q in 0 1; do
    GSMPM_RASTER_TILE_SHARED=$q timeout -k 10 120 python3 bench.py --no-extra-configs --no-cpu-baseline --steps 5 --warmup 2 > $O/q$q.$i.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/q$q.$i.log').read().strip().splitlines()[-1]); print('tile_shared=$q', round(d['render_ms_per_frame'],4), 'ms render;', round(d['ms_per_step'],4), 'ms frame')"
  done
done
