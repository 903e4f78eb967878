# Round 5, GPU call AR: k_fused's grid cap (GSMPM_FUSED_WGS, default the
# resident count 768 = 3 a CU) on bicycle 1M / 256^3, whose ~30,000 chunks
# make every workgroup loop: 768 against 1,536 and 512, interleaved.
set -o pipefail
O=gpurun_out/r05ar
mkdir -p $O
REPS=2 BENCH_ARGS="--config bicycle.json --particles 1000000 --n_grid 256" bash tools/ab_r05.sh $O/ab_D "w768||" "w1536||GSMPM_FUSED_WGS=1536" "w512||GSMPM_FUSED_WGS=512" || exit 1
