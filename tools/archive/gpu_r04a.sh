# Round 4, GPU call A: the GPU suite + smoke, the window-flush micro-benchmark,
# and the render A/B of the hand-written depth order against the library sort.
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
GSMPM_PARITY_OUT=$O/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
tail -22 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 60 ./tools/ubench/window_flush > $O/window_flush.txt 2>&1 && cat $O/window_flush.txt || exit 1
bash tools/ab_env_render.sh GSMPM_RASTER_DSORT own lib $O/ab_dsort > $O/ab_dsort.txt 2>&1; cat $O/ab_dsort.txt
