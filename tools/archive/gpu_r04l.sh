# Round 4, GPU call L: overlapped vs serial render in the bench frame on the
# current render (3 interleaved rounds).
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
for i in 1 2 3; do for ov in 1 0; do
  GSMPM_BENCH_RENDER_OVERLAP=$ov timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > $O/ov_${ov}_$i.json 2> $O/ov_${ov}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/ov_${ov}_$i.json')); print('render_overlap=$ov', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', round(d['render_ms_per_frame'],4))"
done; done | tee $O/ab_overlap.txt
