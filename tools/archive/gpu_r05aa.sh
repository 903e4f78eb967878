# Round 5, GPU call AA: the final tree (after the k_grid_f LDS-DMA records) -- the whole GPU suite, smoke, and the
# two-rank rehearsal line (both ranks on this GPU).
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
GSMPM_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 --multi-configs lego,split \
  > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err || { tail -20 $O/rehearsal_2ranks.err; exit 1; }
tail -1 $O/rehearsal_2ranks.json | cut -c1-400
