# Round 5, GPU call AS: k_fused's grid cap continued -- B' (lego 240,549:
# ~940 full chunks) at 768 against 1,536, and bicycle at 1,536 against 2,304.
set -o pipefail
O=gpurun_out/r05as
mkdir -p $O
REPS=3 BENCH_ARGS="--particles 240549" bash tools/ab_r05.sh $O/ab_Bp "w768||" "w1536||GSMPM_FUSED_WGS=1536" || exit 1
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "w1536||GSMPM_FUSED_WGS=1536" "w2304||GSMPM_FUSED_WGS=2304" || exit 1
