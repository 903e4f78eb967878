# Round 4, GPU call E: the LSD form of the depth order -- its tests (both
# hand-written forms against the library sort), the render A/B of the three
# forms on lego and bicycle, and both render profiles; then the library A/Bs
# of the box-only window zeroing (zbox) and the Newton-refined SVD rsqrt
# (svdnr), and the svdnr long-horizon parity.
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_raster_bwd.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
bash tools/ab_env_render.sh GSMPM_RASTER_DSORT "bucket lsd lib" $O/ab_dsort > $O/ab_dsort.txt 2>&1; cat $O/ab_dsort.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render_D -o run -- python3 tools/render_probe.py > $O/prof_render_D.log 2>&1 || exit 1
cp $(find $O/prof_render_D -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_bicycle.csv && rm -rf $O/prof_render_D
GSMPM_RASTER_DSORT=lsd REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render -o run -- python3 tools/render_probe.py > $O/prof_render.log 2>&1 || exit 1
cp $(find $O/prof_render -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_lego_lsd.csv && rm -rf $O/prof_render
REPS=2 bash tools/ab_libs.sh base zbox svdnr > $O/ab_lego.txt 2>&1 || exit 1
cat $O/ab_lego.txt
BENCH_ARGS="--config lego-fracture.json --material metal" REPS=2 bash tools/ab_libs.sh base svdnr > $O/ab_metal.txt 2>&1 || exit 1
cat $O/ab_metal.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_svdnr.so GSMPM_PARITY_OUT=$O/parity_svdnr timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_long.py -x -q -k "metal or sand" --timeout 280 --timeout-method thread -s > $O/svdnr_parity.log 2>&1
echo "svdnr parity rc $?"
grep -E "passed|failed|substep|Error" $O/svdnr_parity.log | tail -20
