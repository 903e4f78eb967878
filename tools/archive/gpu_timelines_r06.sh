# Per-workgroup timelines on the final round-6 kernels (stamps build):
# k_grid_f's phases, k_fused's phases for jelly and metal.
set -o pipefail
O=gpurun_out/${1:-r06tl}; mkdir -p $O
export GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so
TAG=final timeout -k 10 150 python3 tools/grid_f_phases.py > $O/grid_f_phases.txt 2>&1 || { tail -5 $O/grid_f_phases.txt; exit 1; }
tail -4 $O/grid_f_phases.txt
timeout -k 10 150 python3 tools/wg_timeline_f.py > $O/wg_timeline_jelly.txt 2>&1 || { tail -5 $O/wg_timeline_jelly.txt; exit 1; }
grep -v "^stats" $O/wg_timeline_jelly.txt | head -14
MAT=metal timeout -k 10 150 python3 tools/wg_timeline_f.py > $O/wg_timeline_metal.txt 2>&1 || { tail -5 $O/wg_timeline_metal.txt; exit 1; }
grep -v "^stats" $O/wg_timeline_metal.txt | head -14
