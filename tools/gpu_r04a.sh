# Round 4, first GPU call: the GPU suite + smoke, then A/B of the box-only
# window zeroing (zbox) and the Newton-refined SVD rsqrt (svdnr) on the lego
# bench and the metal config, and the svdnr long-horizon parity (metal, sand).
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
GSMPM_PARITY_OUT=$O/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
tail -22 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
REPS=2 bash tools/ab_libs.sh base zbox svdnr > $O/ab_lego.txt 2>&1 || exit 1
cat $O/ab_lego.txt
BENCH_ARGS="--config lego-fracture.json --material metal" REPS=2 bash tools/ab_libs.sh base svdnr > $O/ab_metal.txt 2>&1 || exit 1
cat $O/ab_metal.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_svdnr.so GSMPM_PARITY_OUT=$O/parity_svdnr timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_long.py -x -q -k "metal or sand" --timeout 500 --timeout-method thread -s > $O/svdnr_parity.log 2>&1
echo "svdnr parity rc $?"
grep -E "passed|failed|substep|Error" $O/svdnr_parity.log | tail -20
