# Round 4, GPU call B: library A/B of the box-only window zeroing (zbox) and
# the Newton-refined SVD rsqrt (svdnr) and the atomic grid accumulator (agrid)
# on the lego bench and the metal config, agrid's parity (MPM + config tests),
# the svdnr long-horizon parity (metal, sand), and a rocprofv3 kernel-stats
# pass of the lego render alone.
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
REPS=2 bash tools/ab_libs.sh base zbox svdnr agrid > $O/ab_lego.txt 2>&1 || exit 1
cat $O/ab_lego.txt
BENCH_ARGS="--config lego-fracture.json --material metal" REPS=2 bash tools/ab_libs.sh base svdnr > $O/ab_metal.txt 2>&1 || exit 1
cat $O/ab_metal.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render -o run -- python3 tools/render_probe.py > $O/prof_render.log 2>&1 || exit 1
cp $(find $O/prof_render -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_lego.csv && rm -rf $O/prof_render
CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_render_D -o run -- python3 tools/render_probe.py > $O/prof_render_D.log 2>&1 || exit 1
cp $(find $O/prof_render_D -name 'run_kernel_stats.csv' | head -n 1) $O/render_kernel_stats_bicycle.csv && rm -rf $O/prof_render_D
python3 tools/dsort_stats.py > $O/dsort_stats.txt 2>&1; cat $O/dsort_stats.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_svdnr.so GSMPM_PARITY_OUT=$O/parity_svdnr timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_long.py -x -q -k "metal or sand" --timeout 500 --timeout-method thread -s > $O/svdnr_parity.log 2>&1
echo "svdnr parity rc $?"
grep -E "passed|failed|substep|Error" $O/svdnr_parity.log | tail -20
