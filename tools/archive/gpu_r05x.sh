# Round 5, GPU call X: k_grid_f with 4 workgroups of 112 lanes a tile
# (GSMPM_GRID_PARTS=4, libgsmpm_p4.so) against 7 of 64 (the product): the
# slab and MPM tests on the variant, then interleaved A/B on lego 100k and
# bicycle 1M.
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_p4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_slab.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=3 bash tools/ab_r05.sh $O/ab_B "cur||" "p4|p4|" || exit 1
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "cur||" "p4|p4|" || exit 1
