# A/B: k_grid_f skipping the v_out store of massless nodes (libgsmpm_skip0.so) vs the default build
set -e
mkdir -p gpurun_out/ab
REPS=3 bash tools/ab_libs.sh base skip0 2>&1 | tee gpurun_out/ab/ab_skip0.txt
