# Round 5, GPU call F: the async-render test, the render A/B with the tighter
# pair capacity, then the profile of the new defaults (bench line, rocprofv3
# kernel stats, PMC passes B and D).
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_raster.py::test_async_forward_matches_workspace_forward > $O/tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|^E " $O/tests.log | head -20
REPS=3 bash tools/ab_r05.sh $O/render "thread||GSMPM_BENCH_RENDER_ASYNC=0" "async||" "async_serial||GSMPM_BENCH_RENDER_OVERLAP=0" "sync_serial||GSMPM_BENCH_RENDER_ASYNC=0 GSMPM_BENCH_RENDER_OVERLAP=0" || exit 1
bash tools/gpu_profile.sh r05f_prof > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -1 gpurun_out/r05f_prof/bench.log | cut -c1-600
