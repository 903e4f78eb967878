# Round 4, GPU call H: the final measurement of the round -- the default bench
# line, its rocprofv3 kernel stats, and the PMC traffic passes for configs B
# and D (tools/gpu_profile.sh), plus the bicycle render's PMC.
set -o pipefail
PMC_RENDER=1 bash tools/gpu_profile.sh r04h > gpurun_out/r04h.log 2>&1
rc=$?
tail -3 gpurun_out/r04h.log
tail -1 gpurun_out/r04h/bench.log
[ $rc -eq 0 ] || exit $rc
# the slab exchange / interior-pass overlap in the eager form (no captured graph: the RCCL group on the comm
# stream, the interior pass on the simulator stream), beside call G's graph trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
pids=""
for r in 0 1; do
  GSMPM_SLAB_GRAPH=0 GSMPM_SHARE_GPU=1 RANK=$r LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29573 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/slabtrace_eager/r$r -o run -- python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/slabtrace_eager_r$r.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -20 $O/slabtrace_eager_r0.log; exit $rc; }
for r in 0 1; do
  f=$(find $O/slabtrace_eager/r$r -name 'run_kernel_trace.csv' | head -n 1)
  python3 tools/overlap_trace.py $f | tee $O/overlap_eager_r$r.txt
done
