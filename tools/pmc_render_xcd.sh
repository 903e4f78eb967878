# FETCH/WRITE of the bicycle render's kernels with the XCD-grouped k_render
# quarters on and off (GSMPM_RASTER_XCD), one --pmc pass per counter.
set -e
O=${1:-gpurun_out/pmc_render_xcd}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=bicycle.json N=1000000 NG=256 REPS=3
for x in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GSMPM_RASTER_XCD=$x timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/x$x$c -o run -- python3 tools/render_probe.py > $O/x$x$c.log 2>&1
    f=$(find $O/x$x$c -name run_counter_collection.csv | head -n 1); cp "$f" $O/x$x.$c.csv; rm -rf $O/x$x$c
  done
done
echo ok
