# Round 4, GPU call U: the digit sort below 4,096 tiles (GSMPM_RASTER_CHUNKED=0)
# -- its test and the lego render A/B against the chunked counting sort.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py -m gpu -x -v --timeout 200 --timeout-method thread -k "below_4096 or digit_tile or depth_order" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
for i in 1 2 3; do for c in 1 0; do
  echo "lego GSMPM_RASTER_CHUNKED=$c $(GSMPM_RASTER_CHUNKED=$c REPS=50 timeout -k 10 120 python3 tools/render_probe.py 2>&1 | tail -n 1)"
done; done | tee $O/ab_chunked.txt
