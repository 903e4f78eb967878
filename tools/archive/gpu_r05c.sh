# Round 5, GPU call C: the outside-chunk lane-order fix (the r05b suite's
# illegal address), the new tests, the LDS banking microbenchmark, then the
# whole GPU suite, smoke and the default bench line.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_mpm.py::test_particles_binned_outside_the_grid" \
  "tests/test_gpu_mpm.py::test_nonfinite_position_reported" "tests/test_gpu_mpm.py::test_heterogeneous_masses" \
  "tests/test_gpu_mpm.py::test_fused_margin_escapes" tests/test_gpu_udon.py > $O/new.log 2>&1
rc=$?
tail -12 $O/new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/ubench/lds_banks > $O/lds_banks.txt 2>&1 && cat $O/lds_banks.txt || exit 1
bash tools/gpu_check.sh r05c
