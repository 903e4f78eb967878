# Round 5, GPU call I: two instances of each captured graph launched in turn
# (a relaunch of one instance waited for its previous launch on the host):
# the MPM GPU tests, the bench A/B against one instance (host call times in
# the .err files), and the frame loop's kernel trace again.
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_bench.py::test_bench_line_contract_and_render_thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit 1
REPS=3 bash tools/ab_r05.sh $O/ab "copies2||GSMPM_BENCH_HOST_TIMING=1" "copies1||GSMPM_GRAPH_COPIES=1 GSMPM_BENCH_HOST_TIMING=1" || exit 1
grep -h "host us" $O/ab/*.err | head -6
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name 'run_kernel_trace.csv' | head -n 1); cp $f $O/frame_trace.csv; rm -rf $O/trace
python3 tools/frame_timeline.py $O/frame_trace.csv | tee $O/frame_timeline.txt
