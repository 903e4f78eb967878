# A/B of the render kernels on one box: bench.py's render_ms_per_frame (the
# frame's render alone, 5 reps) with k_render4 (default) and the per-quarter
# k_render (GSMPM_RASTER_QUARTERS=1), 3 interleaved pairs.
set -e
O=${1:-gpurun_out/ab_render}
mkdir -p $O
for i in 1 2 3; do
  for q in 0 1; do
    GSMPM_RASTER_QUARTERS=$q timeout -k 10 120 python3 bench.py --no-extra-configs --no-cpu-baseline --steps 5 --warmup 2 > $O/q$q.$i.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/q$q.$i.log').read().strip().splitlines()[-1]); print('quarters=$q', round(d['render_ms_per_frame'],4), 'ms render;', round(d['ms_per_step'],4), 'ms frame')"
  done
done
