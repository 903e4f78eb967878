# Round 4, GPU call B: the GPU tests of the new rasterizer sorts and slab
# re-cutting, then the render profiles (rocprofv3 kernel stats, lego and
# bicycle) and the depth-order bucket statistics, library A/B of the box-only
# window zeroing (zbox) and the Newton-refined SVD rsqrt (svdnr) on the lego
# bench and the metal config, and the svdnr long-horizon parity (metal, sand).
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
GSMPM_PARITY_OUT=$O/parity timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_parity_long.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not metal and not ten_frames and not sand_foam and not impulse_window" > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render -o run -- python3 tools/render_probe.py > $O/prof_render.log 2>&1 || exit 1
cp $(find $O/prof_render -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_lego.csv && rm -rf $O/prof_render
CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render_D -o run -- python3 tools/render_probe.py > $O/prof_render_D.log 2>&1 || exit 1
cp $(find $O/prof_render_D -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_bicycle.csv && rm -rf $O/prof_render_D
timeout -k 10 120 python3 tools/dsort_stats.py > $O/dsort_stats.txt 2>&1; cat $O/dsort_stats.txt
bash tools/ab_env_render.sh GSMPM_RASTER_DSORT "own lib" $O/ab_dsort > $O/ab_dsort.txt 2>&1; cat $O/ab_dsort.txt
for i in 1 2; do for ov in 1 0; do
  GSMPM_BENCH_RENDER_OVERLAP=$ov timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > $O/ov_${ov}_$i.json 2> $O/ov_${ov}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/ov_${ov}_$i.json')); print('render_overlap=$ov', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', d['render_ms_per_frame'], d['render_host_ms_per_frame'])"
done; done | tee $O/ab_overlap.txt
