# Round 5, GPU call AT: bicycle's k_fused grid cap at 2,304, 4,608 and
# uncapped (one workgroup a chunk), interleaved.
set -o pipefail
O=gpurun_out/r05at
mkdir -p $O
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "w2304||GSMPM_FUSED_WGS=2304" "w4608||GSMPM_FUSED_WGS=4608" "wall||GSMPM_FUSED_WGS=1000000" || exit 1
