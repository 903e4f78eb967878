# Round 4, GPU call H: the final measurement of the round -- the default bench
# line, its rocprofv3 kernel stats, and the PMC traffic passes for configs B
# and D (tools/gpu_profile.sh), plus the bicycle render's PMC.
set -o pipefail
PMC_RENDER=1 bash tools/gpu_profile.sh r04h > gpurun_out/r04h.log 2>&1
rc=$?
tail -3 gpurun_out/r04h.log
tail -1 gpurun_out/r04h/bench.log
exit $rc
