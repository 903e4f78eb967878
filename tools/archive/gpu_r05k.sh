# Round 5, GPU call K: a 5-round interleaved A/B of the simulator changes on
# the lego bench (sim ms per frame is the figure to read): the previous
# commit's library (head, one graph instance), the current one (k_fused's
# rare arguments behind a pointer, k_grid_f without the slab hooks, packed
# P2G) and the current one with the scalar P2G (nopk).
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
REPS=5 bash tools/ab_r05.sh $O/ab "head|head|GSMPM_GRAPH_COPIES=1" "cur||" "nopk|nopk|" || exit 1
