# Round 4, GPU call G (F again, the refined rsqrt falling back to 1 / sqrtf off
# the normal range, + the owner-grouped window slots A/B): the whole GPU suite + smoke on the new defaults (LSD
# depth order above 262,144 Gaussians, workgroup-per-row digit prefixes, the
# Newton-refined SVD rsqrt), the metal A/B against the exact SVD build, and
# the slab exchange / interior-pass overlap trace (2 RCCL ranks on cuda:0,
# each under its own rocprofv3 kernel trace).
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
for L in libgsmpm.so libgsmpm_svdexact.so; do
  GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/$L timeout -k 10 120 python -u -m pytest tests/test_gpu_constitutive.py -q -k degenerate --timeout 100 --timeout-method thread > $O/svd_degenerate_$L.log 2>&1
  echo "$L degenerate-scale SVD rc $?"; grep -E "passed|failed|^E .*Assertion" $O/svd_degenerate_$L.log | head -4
done
GSMPM_PARITY_OUT=$O/parity timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
tail -22 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
BENCH_ARGS="--config lego-fracture.json --material metal" REPS=2 bash tools/ab_libs.sh base svdexact > $O/ab_metal.txt 2>&1 || exit 1
cat $O/ab_metal.txt
REPS=2 bash tools/ab_libs.sh base owner > $O/ab_owner.txt 2>&1 || exit 1
cat $O/ab_owner.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_owner.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mpm.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/owner_tests.log 2>&1
echo "owner tests rc $?"; tail -2 $O/owner_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
pids=""
for r in 0 1; do
  GSMPM_SHARE_GPU=1 RANK=$r LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/slabtrace/r$r -o run -- python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/slabtrace_r$r.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -20 $O/slabtrace_r0.log; exit $rc; }
for r in 0 1; do
  f=$(find $O/slabtrace/r$r -name 'run_kernel_trace.csv' | head -n 1)
  python3 tools/overlap_trace.py $f | tee $O/overlap_r$r.txt
done
tail -1 $O/slabtrace_r0.log
