# Round 4, GPU call Q: the overlapped render staggered into the next frame
# (bench.py --render-delay-us D), lego bench, 3 interleaved rounds.
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
for i in 1 2 3; do for d in 0 150 400 1000; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 --render-delay-us $d > $O/rd_${d}_$i.json 2> $O/rd_${d}_$i.err || { tail -5 $O/rd_${d}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rd_${d}_$i.json')); print('render_delay_us=$d', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4))"
done; done | tee $O/ab_render_delay.txt
