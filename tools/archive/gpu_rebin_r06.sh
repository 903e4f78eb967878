# Re-binning interval on the round-6 kernels (escapes mark their tiles, XCD
# grouping): lego at R = 20 / 25 / 34 / 50 and metal at 25 / 34 / 50, two rounds.
set -o pipefail
O=gpurun_out/${1:-r06rb}; mkdir -p $O
RS="20 25 34 50" REPS=2 bash tools/rebin_sweep.sh $O/lego > $O/lego.txt 2>&1 || { tail -5 $O/lego.txt; exit 1; }
cat $O/lego.txt
RS="25 34 50" REPS=2 BENCH_ARGS="--config lego-fracture.json --material metal" bash tools/rebin_sweep.sh $O/metal > $O/metal.txt 2>&1 || { tail -5 $O/metal.txt; exit 1; }
cat $O/metal.txt
