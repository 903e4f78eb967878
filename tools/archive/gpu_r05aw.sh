# Round 5, GPU call AW: k_grid_f's grid (7 x min(tiles, GSMPM_GRID_TILES),
# default 1,024: one round of one-wave workgroups) on bicycle 1M, whose
# ~27,600 touched tiles make every workgroup loop: 1,024 against 2,048 and
# 4,096, interleaved.
set -o pipefail
O=gpurun_out/r05aw
mkdir -p $O
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "t1024||" "t2048||GSMPM_GRID_TILES=2048" "t4096||GSMPM_GRID_TILES=4096" || exit 1
