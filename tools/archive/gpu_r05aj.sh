# Round 5, GPU call AJ: k_fused's window store converts two nodes a lane an
# iteration (both nodes' 8 LDS reads behind one wait; GSMPM_STORE_PAIR):
# MPM tests, then interleaved A/B against the previous commit (head) on lego
# 100k (5 rounds) and B' (2).
set -o pipefail
O=gpurun_out/r05aj
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
REPS=5 bash tools/ab_r05.sh $O/ab_B "head|head|" "cur||" || exit 1
REPS=2 BENCH_ARGS="--particles 240549" bash tools/ab_r05.sh $O/ab_Bp "head|head|" "cur||" || exit 1
