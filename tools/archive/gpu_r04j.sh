# Round 4, GPU call J: the pair count published by the depth order's own
# kernels (dsort.h ds_publish) -- raster tests, the render A/B against the
# one-lane publish kernel (GSMPM_RASTER_EARLY_COUNT=0), and the bench line.
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_raster_bwd.py tests/test_gpu_parity_long.py -m gpu -x -v --timeout 200 --timeout-method thread -k "not metal and not ten_frames and not sand_foam and not impulse_window" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
bash tools/ab_env_render.sh GSMPM_RASTER_EARLY_COUNT "1 0" $O/ab_early > $O/ab_early.txt 2>&1; cat $O/ab_early.txt
for i in 1 2; do for ec in 1 0; do
  GSMPM_RASTER_EARLY_COUNT=$ec timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > $O/bench_${ec}_$i.json 2> $O/bench_${ec}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_${ec}_$i.json')); print('early_count=$ec', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', d['render_ms_per_frame'])"
done; done | tee $O/ab_early_bench.txt
