# Re-binning substeps with the grid update forked beside the binning +
# permute (GSMPM_REBIN_FORK, runtime): MPM / config / fold / slab tests with
# the fork, then an interleaved A/B (fork = default, serial = GSMPM_REBIN_FORK=0)
# on B, C, B' and D.
set -o pipefail
O=gpurun_out/${1:-r06rf}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_fold.py tests/test_gpu_slab.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() {  # name env-value args...
  local name=$1 f=$2; shift 2
  GSMPM_REBIN_FORK=$f timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-extra-configs "$@" > $O/${name}.json 2> $O/${name}.err || { tail -5 $O/${name}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${name}.json')); print('$name', round(d['value']/1e9,4), 'ms/frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), d['kernels_ms_per_launch'])"
}
for rep in 1 2 3; do
  for v in fork serial; do
    f=1; [ $v = serial ] && f=0
    run B_${v}_$rep $f --steps 20 --warmup 3 || exit 1
    run C_${v}_$rep $f --steps 20 --warmup 3 --config lego-fracture.json --material metal || exit 1
    run Bp_${v}_$rep $f --steps 10 --warmup 3 --particles 240549 || exit 1
    [ $rep -le 2 ] && { run D_${v}_$rep $f --steps 4 --warmup 2 --config bicycle.json --particles 1000000 --n_grid 256 || exit 1; }
  done
done
