# Round 4, GPU call O: the overlapped render on its own CUs (bench.py
# --render-cus N: the simulator's and the render's streams on disjoint CU
# masks) against both streams on every CU, lego bench, 3 interleaved rounds.
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
for i in 1 2 3; do for rc in 0 16 32 64; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 --render-cus $rc > $O/rc_${rc}_$i.json 2> $O/rc_${rc}_$i.err || { tail -5 $O/rc_${rc}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rc_${rc}_$i.json')); print('render_cus=$rc', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', round(d['render_ms_per_frame'],4), d['config'].get('render_cus'))"
done; done | tee $O/ab_render_cus.txt
