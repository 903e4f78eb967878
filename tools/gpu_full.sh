set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 > gpurun_out/v1/tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/v1/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/v1/bench.log 2>&1
