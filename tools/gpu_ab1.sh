set -e
mkdir -p gpurun_out/ab
bash tools/ab_env_render_wgs.sh 2>&1 | tee gpurun_out/ab/ab_render_wgs.txt
bash tools/ab_skip0.sh
