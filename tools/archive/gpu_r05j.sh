# Round 5, GPU call J: k_fused's rare arguments behind one device pointer (SGPR
# spills 89 -> 42), packed-f32 P2G, two graph instances in turn: the whole GPU
# suite, then the bench A/B against the previous commit's library (head), the
# scalar P2G (nopk) and one graph instance (copies1), then the frame trace.
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=3 bash tools/ab_r05.sh $O/ab "new||" "head|head|" "nopk|nopk|" "copies1||GSMPM_GRAPH_COPIES=1" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name 'run_kernel_trace.csv' | head -n 1); cp $f $O/frame_trace.csv; rm -rf $O/trace
python3 tools/frame_timeline.py $O/frame_trace.csv | tee $O/frame_timeline.txt
