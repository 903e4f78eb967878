# Round 5, GPU call AE: k_render with 2 and 1 list entries a lane a batch
# (GSMPM_RENDER_Q; LDS 5 / 2.5 KB against 10: room beside three k_fused
# workgroups' 152 KB, so the overlapped render can share their CUs):
# raster tests on q2, the render alone (lego), and the bench frame A/B.
set -o pipefail
O=gpurun_out/r05ae
mkdir -p $O
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_q2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_raster.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for L in cur q2 q1; do
    if [ $L = cur ]; then LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$L.so; fi
    GSMPM_LIB=$LIB REPS=50 timeout -k 10 120 python3 tools/render_probe.py > $O/lego.$L.$i.log 2>&1 || { tail -5 $O/lego.$L.$i.log; exit 1; }
    echo "lego $L $(tail -n 1 $O/lego.$L.$i.log)"
  done
done | tee $O/render_alone.txt
REPS=3 bash tools/ab_r05.sh $O/ab "cur||" "q2|q2|" "q1|q1|" || exit 1
