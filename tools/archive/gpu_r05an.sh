# Round 5, GPU call AN: the final tree as the driver runs it -- the whole GPU
# suite, smoke, and the default bench line (traffic filled from the committed
# PMC summaries of this source).
set -o pipefail
O=gpurun_out/r05an
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']/1e9,4), d['ms_per_step'], r['frac'], r['traffic'], r['traffic_frac'], d['cpu_baseline']['value'])"
