# One GPU call of round 6: optional test selection, then bench lines.  Every
# step has its own time limit and the steps are chained with && (a fault,
# abort or timeout ends the call).  Usage:
#   bash tools/gpu_r06.sh <tag> "<pytest args or -> " "<bench args or -> " [rocprof 0|1]
set -o pipefail
TAG=$1; TESTS=${2:--}; BENCH=${3:--}; PROF=${4:-0}
O=gpurun_out/$TAG
mkdir -p $O
run_tests() {
  [ "$TESTS" = "-" ] && return 0
  timeout -k 10 1000 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  local rc=$?; tail -3 $O/tests.log; return $rc
}
run_bench() {
  [ "$BENCH" = "-" ] && return 0
  timeout -k 10 400 python3 bench.py $BENCH > $O/bench.log 2>&1
  local rc=$?; tail -c 400 $O/bench.log; echo; return $rc
}
run_prof() {
  [ "$PROF" = "0" ] && return 0
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-extra-configs --no-cpu-baseline --steps 50 --warmup 5 > $O/prof.log 2>&1
  local rc=$?
  f=$(find $O/prof -name 'run_kernel_stats.csv' | head -n 1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv
  f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1); [ -n "$f" ] && python3 tools/trace_summary.py "$f" > $O/trace_summary.txt
  rm -rf $O/prof; return $rc
}
run_tests && run_bench && run_prof && echo "ALL OK"
