# Round 5, GPU call B: the round's new tests first (non-finite flag, heterogeneous
# masses, the LSD overflow fallback, the depth-order cases), then the whole GPU
# suite, smoke and the default bench line.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_mpm.py::test_nonfinite_position_reported" "tests/test_gpu_mpm.py::test_heterogeneous_masses" \
  "tests/test_gpu_raster.py::test_depth_bucket_overflow_takes_lsd_fallback" \
  "tests/test_gpu_raster.py::test_depth_order_matches_library_sort" > $O/new.log 2>&1
rc=$?
tail -12 $O/new.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh r05b
