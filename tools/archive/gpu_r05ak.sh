# Round 5, GPU call AK: config C (metal, 500 substeps) with the spread of 10
# permuted-order oracles instead of 3 (GSMPM_SPREAD_RUNS=10): the GPU's
# F_trial error against a better-sampled spread of the reference's valid
# outputs (the round-4 verdict's weak item 1).
set -o pipefail
O=gpurun_out/r05ak
mkdir -p $O
GSMPM_SPREAD_RUNS=10 GSMPM_PARITY_OUT=$O/parity timeout -k 10 900 python -u -m pytest -x -v -s --timeout 850 --timeout-method thread tests/test_gpu_parity_long.py -k "config_C_metal" > $O/c10.log 2>&1
rc=$?; tail -3 $O/c10.log; grep -E "^E " $O/c10.log | head -5; exit $rc
