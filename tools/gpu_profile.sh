# One GPU call: bench line, rocprofv3 kernel stats of the bench, PMC passes
# for config B (lego, tools/pmc.sh) and config D (bicycle, tools/pmc_D.sh).
# Raw traces are pruned at the end so gpurun_out/ stays small (only the
# summaries travel back).  Usage: bash tools/gpu_profile.sh <tag>
set -e
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-extra-configs --no-cpu-baseline --steps 20 --warmup 5 > $O/prof.log 2>&1
f=$(find $O/prof -name 'run_kernel_stats.csv' | head -n 1)
cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1
  for d in p1 p2 p3 p4; do rm -rf $O/pmc/$d; done
  bash tools/pmc_D.sh $O/pmcD > $O/pmcD.log 2>&1
  if [ "${PMC_RENDER:-0}" = "1" ]; then bash tools/pmc_render_D.sh $O/pmc_render_D > $O/pmc_render_D.log 2>&1; fi
fi
echo ok
