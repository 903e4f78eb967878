# Round 5, GPU call D: LDS banking microbenchmark; the outside-grid test under
# the library variants (which change moved x?); the round's new tests; then
# the whole GPU suite without -x (the full picture in one call).
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 60 tools/ubench/lds_banks > $O/lds_banks.txt 2>&1; cat $O/lds_banks.txt
T="tests/test_gpu_mpm.py::test_particles_binned_outside_the_grid"
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread $T > $O/outside_$n.log 2>&1
  echo "outside[$n] rc=$? $(grep -E 'passed|failed' $O/outside_$n.log | tail -1) $(grep -o "AssertionError: .*" $O/outside_$n.log | head -1)"
}
run default
run norec GSMPM_COVER_RECORDS=0
run b96 GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_b96.so
run r04 GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_r04.so
run r04norebin GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_r04.so GSMPM_LANE_BALANCE=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "suite rc=$?"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -25
