# rocprofv3 kernel stats of the render alone (GPU box): bash tools/render_prof.sh <tag>
set -e
O=gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 tools/render_probe.py > $O/plain.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/render_probe.py > $O/prof.log 2>&1
cp $(find $O/prof -name "run_kernel_stats.csv" | head -n 1) $O/stats.csv
rm -rf $O/prof
