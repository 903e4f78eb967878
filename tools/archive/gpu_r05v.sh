# Round 5, GPU call V: k_grid_f's extra-chunk reads batched (second chunks of
# the covering tiles as two batches of 4, saddr slot loads, first record in
# LDS before the tile loop, dt*gravity from the host): MPM GPU tests, then
# interleaved A/B against the previous commit (head) on lego 100k (B),
# lego 240,549 (B') and bicycle 1M / 256^3 on one GPU.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_goldens.py tests/test_gpu_slab.py tests/test_gpu_parity_long.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=3 bash tools/ab_r05.sh $O/ab_B "head|head|" "cur||" || exit 1
REPS=2 BENCH_ARGS="--particles 240549" bash tools/ab_r05.sh $O/ab_Bp "head|head|" "cur||" || exit 1
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "head|head|" "cur||" || exit 1
