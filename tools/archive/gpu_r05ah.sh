# Round 5, GPU call AH: where the overlapped render runs inside the frame
# (rocprofv3 kernel trace of the lego bench at --rebin 20 and 50,
# tools/render_placement.py).
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for R in 20 50; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr$R -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 --rebin $R > $O/b$R.log 2>&1 || { tail -5 $O/b$R.log; exit 1; }
  f=$(find $O/tr$R -name 'run_kernel_trace.csv' | head -n 1)
  python3 tools/render_placement.py "$f" > $O/placement_r$R.txt 2>&1 || { tail -5 $O/placement_r$R.txt; exit 1; }
  rm -rf $O/tr$R
done
cat $O/placement_r20.txt $O/placement_r50.txt
