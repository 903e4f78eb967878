# Round 5, GPU call AY: stress-bearing materials re-bin every 20 substeps
# (was 10): the MPM, configs, constitutive, udon and long-horizon parity
# tests, then the PMC passes for the new sources (B, D, C, B') and the
# default bench line with rocprofv3 kernel stats.
set -o pipefail
O=gpurun_out/r05ay
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_constitutive.py tests/test_gpu_udon.py tests/test_gpu_parity_long.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 900 bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
for d in p1 p2 p3 p4; do rm -rf $O/pmc/$d; done
timeout -k 10 900 bash tools/pmc_D.sh $O/pmcD > $O/pmcD.log 2>&1 || { tail -5 $O/pmcD.log; exit 1; }
CONFIG=lego-fracture.json N=100000 NG=128 MAT=metal timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcC C > $O/pmcC.log 2>&1 || { tail -5 $O/pmcC.log; exit 1; }
CONFIG=lego.json N=240549 NG=128 timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcBp Bp > $O/pmcBp.log 2>&1 || { tail -5 $O/pmcBp.log; exit 1; }
echo pmc ok
