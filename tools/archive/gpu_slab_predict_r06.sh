# Slab predictions (tools/slab_predict.py) re-measured on the final round-6
# kernels: config D and the lego headline.
set -o pipefail
O=gpurun_out/${1:-r06sp}; mkdir -p $O
timeout -k 10 500 python3 tools/slab_predict.py --out $O/slab_prediction_D.json > $O/D.log 2>&1 || { tail -20 $O/D.log; exit 1; }
tail -6 $O/D.log
timeout -k 10 300 python3 tools/slab_predict.py --config lego.json --particles 100000 --n_grid 128 --out $O/slab_prediction_lego.json > $O/lego.log 2>&1 || { tail -20 $O/lego.log; exit 1; }
tail -6 $O/lego.log
