# Round 5, GPU call R: k_grid_f node_reads with every LDS read first (no branches around them):
# box, lane order and the chunk count) as one inline-asm round trip: MPM +
# config + slab GPU tests, then a 5-round A/B against the previous commit
# (head).
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_slab.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=5 bash tools/ab_r05.sh $O/ab "head|head|" "cur||" || exit 1
