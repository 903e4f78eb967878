# k_fused / k_grid_f limiter passes (GPU box): bash tools/pmc2.sh <outdir> "<counters pass1>" "<counters pass2>" ...
set -e
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for cs in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $OUT/q$i -o run -- python3 tools/pmc_probe.py > $OUT/q$i.log 2>&1
  f=$(find $OUT/q$i -name run_counter_collection.csv | head -n 1); cp "$f" $OUT/q$i.csv; rm -rf $OUT/q$i
done
echo ok
