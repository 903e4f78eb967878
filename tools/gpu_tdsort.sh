# per-tile depth sort: raster parity tests, then the lego render alone with it off / on (3 interleaved rounds)
set -e
mkdir -p gpurun_out/td
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_raster_bwd.py tests/test_gpu_goldens.py tests/test_gpu_main_e2e.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/td/tests.log 2>&1 || { tail -40 gpurun_out/td/tests.log; exit 1; }
tail -2 gpurun_out/td/tests.log
for i in 1 2 3; do
  for TD in 0 1; do
    GSMPM_RASTER_TILE_DSORT=$TD REPS=50 timeout -k 10 120 python3 tools/render_probe.py > gpurun_out/td/lego.$TD.$i.log 2>&1
    echo "lego tile_dsort=$TD $(tail -n 1 gpurun_out/td/lego.$TD.$i.log)"
  done
done
for i in 1 2; do
  for TD in 0 1; do
    GSMPM_RASTER_TILE_DSORT=$TD timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > gpurun_out/td/bench.$TD.$i.json 2> gpurun_out/td/bench.$TD.$i.err
    python3 -c "import json; d=json.load(open('gpurun_out/td/bench.$TD.$i.json')); print('bench tile_dsort=$TD', round(d['value']/1e9,4), 'frame', round(d['ms_per_step'],4), 'sim', round(d['sim_ms_per_frame'],4), 'render', round(d['render_ms_per_frame'],4))"
  done
done
