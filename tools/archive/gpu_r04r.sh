# Round 4, GPU call R: the previous frame's render submitted before the next
# frame's graph (bench.py --render-first 1) against after it, lego bench, 3
# interleaved rounds; then one kernel trace of --render-first 1.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
for i in 1 2 3; do for rf in 0 1; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 --render-first $rf > $O/rf_${rf}_$i.json 2> $O/rf_${rf}_$i.err || { tail -5 $O/rf_${rf}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rf_${rf}_$i.json')); print('render_first=$rf', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4))"
done; done | tee $O/ab_render_first.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 --render-first 1 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name 'run_kernel_trace.csv' | head -n 1); cp $f $O/frame_trace.csv; rm -rf $O/trace
python3 tools/frame_timeline.py $O/frame_trace.csv | tee $O/frame_timeline.txt
