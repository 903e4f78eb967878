# Round 5, GPU call E: the fixed / new tests (outside-grid, weighted re-cut,
# async render), then interleaved A/B of the k_fused / k_grid_f changes on the
# lego bench (3 rounds), then the async render against the render thread.
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_mpm.py::test_particles_binned_outside_the_grid tests/test_gpu_mpm.py::test_heterogeneous_masses \
  tests/test_gpu_slab.py::test_gpu_slabs_weighted_recut tests/test_gpu_raster.py::test_async_forward_matches_workspace_forward \
  > $O/tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|Error" $O/tests.log | head -20
REPS=3 BENCH_ARGS="--render-async 0" bash tools/ab_r05.sh $O/ab "v4k|v4k|GSMPM_COVER_RECORDS=0" "v4kmass|v4kmass|GSMPM_COVER_RECORDS=0" \
  "b128dpp||GSMPM_COVER_RECORDS=0" "default||" "nt|nt|" || exit 1
REPS=3 bash tools/ab_r05.sh $O/render "thread||GSMPM_BENCH_RENDER_ASYNC=0" "async||" "async_serial||GSMPM_BENCH_RENDER_OVERLAP=0" || exit 1
