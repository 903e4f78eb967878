# Round 5, GPU call Y: k_fused's workgroups take the chunks in a size-ranked
# snake order (ChunkOut.cslot, k_finish_bins): MPM GPU tests, then
# interleaved A/B on lego 100k: head (commit e07a694), cur, and cur with
# GSMPM_CHUNK_ORDER=0 (the same library in chunk order); bicycle 1M and B'.
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_goldens.py tests/test_gpu_slab.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=3 bash tools/ab_r05.sh $O/ab_B "head|head|" "cur||" "off||GSMPM_CHUNK_ORDER=0" || exit 1
REPS=2 BENCH_ARGS="--particles 240549" bash tools/ab_r05.sh $O/ab_Bp "head|head|" "cur||" || exit 1
REPS=1 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "head|head|" "cur||" || exit 1
