# The SIMD of each k_fused workgroup's wave 0 (stamps build, lego jelly)
set -o pipefail
O=gpurun_out/${1:-r06simd}; mkdir -p $O
export GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so
timeout -k 10 150 python3 tools/wg_timeline_f.py > $O/wg_timeline_jelly.txt 2>&1 || { tail -5 $O/wg_timeline_jelly.txt; exit 1; }
grep -E "SIMD|CUs used|CU load" $O/wg_timeline_jelly.txt
