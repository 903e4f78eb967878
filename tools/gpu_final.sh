# One GPU call: the GPU test suite, smoke, then the profile set (bench line, rocprofv3 stats, PMC) under <tag>
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 && \
tail -2 gpurun_out/$TAG/tests.log && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 && \
tail -1 gpurun_out/$TAG/smoke.log && \
bash tools/gpu_profile.sh $TAG
