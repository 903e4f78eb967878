# Round 6's final measurement set (one GPU call): the bench line, rocprofv3
# kernel stats + per-kernel trace summary of the bench, and PMC FETCH_SIZE /
# WRITE_SIZE / SQ passes for configs B, B', C (metal) and D, each pass its own
# --pmc run.  Output under gpurun_out/<tag>/.  Usage: bash tools/gpu_final_r06.sh <tag>
set -o pipefail
TAG=${1:-r06final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit 1
tail -c 300 $O/bench.log; echo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-extra-configs --no-cpu-baseline --steps 50 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/kernel_stats.csv
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1); python3 tools/trace_summary.py "$f" > $O/trace_summary.txt
grep -v "^{" $O/prof.log | tail -2; grep "^{" $O/prof.log > $O/prof_bench.json
rm -rf $O/prof
CONFIG=lego.json N=100000 NG=128 bash tools/pmc_cfg.sh $O/pmcB B > $O/pmcB.log 2>&1 || exit 1
CONFIG=lego.json N=240549 NG=128 bash tools/pmc_cfg.sh $O/pmcBp Bp > $O/pmcBp.log 2>&1 || exit 1
CONFIG=lego-fracture.json N=100000 NG=128 MAT=metal bash tools/pmc_cfg.sh $O/pmcC C > $O/pmcC.log 2>&1 || exit 1
CONFIG=bicycle.json N=1000000 NG=256 bash tools/pmc_cfg.sh $O/pmcD D > $O/pmcD.log 2>&1 || exit 1
for d in pmcB pmcBp pmcC pmcD; do rm -rf $O/$d/p1.csv $O/$d/p3.csv $O/$d/p4.csv; done
echo "ALL OK"
