# Round 5, GPU call BB: the stress-bearing re-binning interval continued
# (default 20 now) on config C (lego-fracture, metal) as the
# bench main workload: 20 against 25 and 30, interleaved.
set -o pipefail
O=gpurun_out/r05bb
mkdir -p $O
for rep in 1 2 3; do
  for R in 20 25 30; do
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 --config lego-fracture.json --material metal --rebin $R > $O/r${R}_$rep.json 2> $O/r${R}_$rep.err || { echo "FAIL $R"; tail -5 $O/r${R}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r${R}_$rep.json')); k=d['kernels_ms_per_launch']; print('rebin $R', round(d['value']/1e9,4), 'frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'k_fused', round(k['k_fused']*1e3,2), 'binning/frame', round(d['kernels_ms_per_frame']['binning'],4))" | tee -a $O/summary.txt
  done
done
