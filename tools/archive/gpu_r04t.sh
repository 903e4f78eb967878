# Round 4, GPU call T: the final validation and measurement of the round --
# the whole GPU suite + smoke, then the bench line, its rocprofv3 kernel
# stats and the PMC traffic passes (tools/gpu_profile.sh).
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
GSMPM_PARITY_OUT=$O/parity timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
bash tools/gpu_profile.sh r04t_prof > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -1 gpurun_out/r04t_prof/bench.log
