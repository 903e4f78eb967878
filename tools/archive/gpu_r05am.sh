# Round 5, GPU call AM: per-workgroup timelines of the final kernels (stamps
# build): k_grid_f's phases with the records by LDS-DMA, k_fused's phases,
# and the kernel boundaries.
set -o pipefail
O=gpurun_out/r05am
mkdir -p $O
export GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so
TAG=final timeout -k 10 150 python3 tools/grid_f_phases.py > $O/grid_f_phases.txt 2>&1 || { tail -5 $O/grid_f_phases.txt; exit 1; }
tail -1 $O/grid_f_phases.txt
timeout -k 10 150 python3 tools/wg_timeline_f.py > $O/wg_timeline_f.txt 2>&1 || { tail -5 $O/wg_timeline_f.txt; exit 1; }
grep -v "^stats" $O/wg_timeline_f.txt | head -12
