# XCD-affine chunk order (k_chunk_order_xcd, GSMPM_CHUNK_XCD): the MPM,
# config and slab tests on the new default, then an interleaved A/B against
# the size order alone (cx0) on B, C and B'.
set -o pipefail
O=gpurun_out/${1:-r06cx}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_slab.py tests/test_gpu_fold.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
VARIANTS="base cx0" CONFIGS="B C Bp" REPS=3 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
