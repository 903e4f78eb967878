# Round 5, GPU call H: the LDS banking microbenchmark with inline-asm b128
# reads and partial-exec lane groups; a kernel trace of the bench frame loop
# (which render kernels slow the simulator beside them); the tile sort's
# block-radix-sort form (smaller LDS) against the default in the frame.
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 60 tools/ubench/lds_banks > $O/lds_banks.txt 2>&1 || { cat $O/lds_banks.txt; exit 1; }
cat $O/lds_banks.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name 'run_kernel_trace.csv' | head -n 1); cp $f $O/frame_trace.csv; rm -rf $O/trace
python3 tools/frame_timeline.py $O/frame_trace.csv | tee $O/frame_timeline.txt
REPS=3 bash tools/ab_r05.sh $O/ab "default||" "brs||GSMPM_TILE_BRS=1" || exit 1
