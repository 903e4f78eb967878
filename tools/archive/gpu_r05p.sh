# Round 5, GPU call P: the final tree's profile -- bench line, rocprofv3
# kernel stats, PMC passes for configs B and D (tools/gpu_profile.sh), and
# k_grid_f's per-workgroup phases (stamps build).
set -o pipefail
bash tools/gpu_profile.sh r05_final > gpurun_out/r05_final_profile.log 2>&1 || { tail -20 gpurun_out/r05_final_profile.log; exit 1; }
tail -1 gpurun_out/r05_final/bench.log | cut -c1-700
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so TAG=final timeout -k 10 150 python3 tools/grid_f_phases.py > gpurun_out/r05_final/grid_f_phases.txt 2>&1 || { tail -5 gpurun_out/r05_final/grid_f_phases.txt; exit 1; }
tail -1 gpurun_out/r05_final/grid_f_phases.txt
