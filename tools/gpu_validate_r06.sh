# Round-end validation on one GPU: the whole -m gpu suite, smoke(), and the
# default bench line (which now carries the committed PMC traffic).
# Usage: bash tools/gpu_validate_r06.sh <tag>; output under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-r06v}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -30 $O/gpu_suite.txt; exit 1; }
tail -3 $O/gpu_suite.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600])"
echo "ALL OK"
