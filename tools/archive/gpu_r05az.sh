# Round 5, GPU call AZ: the final tree (stress-bearing re-binning at 20) as the driver runs it: the
# default bench line and rocprofv3 kernel stats (tools/gpu_profile.sh without
# PMC: the traffic files are this source's), the whole GPU suite and smoke.
set -o pipefail
O=gpurun_out/r05az
mkdir -p $O
PMC=0 timeout -k 10 700 bash tools/gpu_profile.sh r05az > $O/profile.log 2>&1 || { tail -5 $O/profile.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
