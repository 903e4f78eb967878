# Round 5, GPU call AB: cover records on grids past kFuseTiles (k_cover_records
# after k_scan_tiles: config D's 256^3), so D's k_grid_f takes the record
# path with the LDS-DMA prefetch instead of the tile tables: MPM / slab /
# configs GPU tests, then interleaved A/B against commit 036abf2 (head) on
# bicycle 1M / 256^3 and lego 100k.
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_configs.py tests/test_gpu_mpm.py tests/test_gpu_parity_long.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "head|head|" "cur||" || exit 1
REPS=2 bash tools/ab_r05.sh $O/ab_B "head|head|" "cur||" || exit 1
