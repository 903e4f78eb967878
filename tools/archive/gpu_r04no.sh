# Round 4, GPU call N (+ call O appended): what the render costs inside the bench frame -- the
# lego bench with and without the render (3 interleaved rounds); and one
# rocprofv3 kernel trace of the overlapped frame loop for the timeline.
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
for i in 1 2 3; do for nr in 0 1; do
  a=""; [ $nr -eq 1 ] && a="--no-render"
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 $a > $O/nr_${nr}_$i.json 2> $O/nr_${nr}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/nr_${nr}_$i.json')); print('no_render=$nr', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4))"
done; done | tee $O/ab_norender.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-extra-configs --steps 6 --warmup 2 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name 'run_kernel_trace.csv' | head -n 1); cp $f $O/frame_trace.csv; rm -rf $O/trace
python3 tools/frame_timeline.py $O/frame_trace.csv | tee $O/frame_timeline.txt

cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
for i in 1 2 3; do for rc in 0 16 32 64; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 --render-cus $rc > $O/rc_${rc}_$i.json 2> $O/rc_${rc}_$i.err || { tail -5 $O/rc_${rc}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rc_${rc}_$i.json')); print('render_cus=$rc', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', round(d['render_ms_per_frame'],4), d['config'].get('render_cus'))"
done; done | tee $O/ab_render_cus.txt
