# Round 5, GPU call AU: k_fused's grid cap scaled by the scene's rounds of
# full chunks (<= 6): MPM / configs / slab tests, then bicycle 1M at the new
# default (5 rounds) against GSMPM_FUSED_WGS=768 (the old one round), and a
# lego check (its cap is unchanged).  Then the PMC passes for the new sources
# (B, D, C, B').
set -o pipefail
O=gpurun_out/r05au
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_slab.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "old||GSMPM_FUSED_WGS=768" "new||" || exit 1
REPS=2 bash tools/ab_r05.sh $O/ab_B "old||GSMPM_FUSED_WGS=768" "new||" || exit 1
timeout -k 10 900 bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
timeout -k 10 900 bash tools/pmc_D.sh $O/pmcD > $O/pmcD.log 2>&1 || { tail -5 $O/pmcD.log; exit 1; }
CONFIG=lego-fracture.json N=100000 NG=128 MAT=metal timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcC C > $O/pmcC.log 2>&1 || { tail -5 $O/pmcC.log; exit 1; }
CONFIG=lego.json N=240549 NG=128 timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcBp Bp > $O/pmcBp.log 2>&1 || { tail -5 $O/pmcBp.log; exit 1; }
for d in p1 p2 p3 p4; do rm -rf $O/pmc/$d; done
echo pmc ok
