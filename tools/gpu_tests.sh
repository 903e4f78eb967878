# the GPU test suite and smoke under <tag> (no profile)
set -o pipefail
TAG=${1:-v}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=10 > gpurun_out/$TAG/tests.log 2>&1 && \
tail -14 gpurun_out/$TAG/tests.log && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 && \
tail -1 gpurun_out/$TAG/smoke.log
