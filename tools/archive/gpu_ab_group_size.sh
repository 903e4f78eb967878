# k_grid_f XCD group size (GSMPM_GRID_GROUP; the chunk order follows it):
# base 16 vs 8 vs 32 on B, B', D; 2 interleaved rounds.
set -o pipefail
O=gpurun_out/${1:-r06gs}; mkdir -p $O
VARIANTS="base g8 g32" CONFIGS="B Bp D" REPS=2 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
