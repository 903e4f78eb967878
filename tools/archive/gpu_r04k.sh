# Round 4, GPU call K: k_dsort_big only when a bucket exceeds 256 entries --
# the raster tests (depth-order cases: layered = workgroup sort, flat =
# overflow fallback) and the render timing.
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_raster_bwd.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
bash tools/ab_env_render.sh GSMPM_RASTER_EARLY_COUNT "1 0" $O/ab_early > $O/ab_early.txt 2>&1; cat $O/ab_early.txt
timeout -k 10 120 python3 tools/dsort_stats.py > $O/dsort_stats.txt 2>&1; cat $O/dsort_stats.txt
