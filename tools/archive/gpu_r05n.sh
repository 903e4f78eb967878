# Round 5, GPU call N: the next-chunk prefetch of k_fused kept as unwaited
# vector loads (matters when a workgroup owns several chunks: config D):
# MPM tests, then A/B against the previous commit on lego (3 rounds) and on
# bicycle 1M / 256^3 (2 rounds).
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=3 bash tools/ab_r05.sh $O/ab "head|head|" "cur||" || exit 1
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/abD "headD|head|" "curD||" || exit 1
