# rocprofv3 kernel stats of the other BASELINE configs on the final round-6
# kernels: B' (240,549), C (lego-fracture metal), D (bicycle 1M / 256^3).
set -o pipefail
O=gpurun_out/${1:-r06pc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # tag args...
  local t=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py --no-extra-configs --no-cpu-baseline "$@" > $O/prof_$t.log 2>&1 || { tail -5 $O/prof_$t.log; exit 1; }
  f=$(find $O/prof_$t -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/kernel_stats_$t.csv
  f=$(find $O/prof_$t -name 'run_kernel_trace.csv' | head -n 1); python3 tools/trace_summary.py "$f" > $O/trace_summary_$t.txt
  grep "^{" $O/prof_$t.log > $O/bench_$t.json; rm -rf $O/prof_$t
  head -6 $O/trace_summary_$t.txt
}
prof Bp --steps 10 --warmup 3 --particles 240549 || exit 1
prof C --steps 20 --warmup 3 --config lego-fracture.json --material metal || exit 1
prof D --steps 4 --warmup 2 --config bicycle.json --particles 1000000 --n_grid 256 || exit 1
