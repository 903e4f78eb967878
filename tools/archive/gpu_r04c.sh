# Round 4, GPU call C: library A/B of the box-only window zeroing (zbox) and
# the Newton-refined SVD rsqrt (svdnr) on the lego bench and the metal config,
# and the svdnr long-horizon parity (metal, sand).
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
REPS=2 bash tools/ab_libs.sh base zbox svdnr > $O/ab_lego.txt 2>&1 || exit 1
cat $O/ab_lego.txt
BENCH_ARGS="--config lego-fracture.json --material metal" REPS=2 bash tools/ab_libs.sh base svdnr > $O/ab_metal.txt 2>&1 || exit 1
cat $O/ab_metal.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_svdnr.so GSMPM_PARITY_OUT=$O/parity_svdnr timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_long.py -x -q -k "metal or sand" --timeout 400 --timeout-method thread -s > $O/svdnr_parity.log 2>&1
echo "svdnr parity rc $?"
grep -E "passed|failed|substep|Error" $O/svdnr_parity.log | tail -20
