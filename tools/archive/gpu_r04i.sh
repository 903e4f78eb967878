# Round 4, GPU call I: the 8,192-pair LSD chunks (GSMPM_RASTER_LSD_I=32) --
# raster tests and the render A/B -- and the PMC traffic passes of configs B
# and D on the current simulator sources.
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
bash tools/ab_env_render.sh GSMPM_RASTER_LSD_I "16 32" $O/ab_lsd_i > $O/ab_lsd_i.txt 2>&1; cat $O/ab_lsd_i.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1 || exit 1
for d in p1 p2 p3 p4; do rm -rf $O/pmc/$d; done
bash tools/pmc_D.sh $O/pmcD > $O/pmcD.log 2>&1 || exit 1
python3 -c "import json; [print(f, json.load(open(f))['source_sha']) for f in ('$O/pmc/traffic.json', '$O/pmcD/traffic_D.json')]"
