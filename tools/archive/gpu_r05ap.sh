# Round 5, GPU call AP: PMC traffic of configs C (lego-fracture metal) and
# B' (lego 240,549) on the final sources, so the bench line's other configs
# carry traffic_frac too; then the default bench line to check it.
set -o pipefail
O=gpurun_out/r05ap
mkdir -p $O
CONFIG=lego-fracture.json N=100000 NG=128 MAT=metal timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcC C > $O/pmcC.log 2>&1 || { tail -5 $O/pmcC.log; exit 1; }
CONFIG=lego.json N=240549 NG=128 timeout -k 10 600 bash tools/pmc_cfg.sh $O/pmcBp Bp > $O/pmcBp.log 2>&1 || { tail -5 $O/pmcBp.log; exit 1; }
python3 -c "import json; [print(t, {k: round(v['bytes_per_launch']/1e6,2) for k,v in json.load(open('$O/pmc'+t+'/traffic_'+t+'.json'))['kernels'].items()}) for t in ('C','Bp')]"
