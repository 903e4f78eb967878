# Round 5, GPU call T: k_render (ids / keys raw, tested a batch later) + k_tile_hist and
# k_tile_scatter with their loads batched (tile totals, keys, chunk offsets):
# raster GPU tests, the render alone (lego, bicycle; previous
# commit = head), and the bench frame A/B.
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_raster.py tests/test_gpu_udon.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
for i in 1 2 3; do
  for L in head cur; do
    if [ $L = head ]; then LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_head.so; else LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; fi
    GSMPM_LIB=$LIB REPS=50 timeout -k 10 120 python3 tools/render_probe.py > $O/lego.$L.$i.log 2>&1 || { tail -5 $O/lego.$L.$i.log; exit 1; }
    echo "lego $L $(tail -n 1 $O/lego.$L.$i.log)"
    GSMPM_LIB=$LIB CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 python3 tools/render_probe.py > $O/bicycle.$L.$i.log 2>&1 || { tail -5 $O/bicycle.$L.$i.log; exit 1; }
    echo "bicycle $L $(tail -n 1 $O/bicycle.$L.$i.log)"
  done
done | tee $O/render_alone.txt
REPS=3 bash tools/ab_r05.sh $O/ab "head|head|" "cur||" || exit 1
