# Round 5, GPU call U: per-workgroup timelines after the G2P staging fix
# (stamps build): k_fused phases, kernel boundaries.
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so
timeout -k 10 150 python3 tools/wg_timeline_f.py > $O/wg_timeline_f.txt 2>&1 || { tail -5 $O/wg_timeline_f.txt; exit 1; }
cat $O/wg_timeline_f.txt | grep -v "^stats"
timeout -k 10 150 python3 tools/boundary_gaps.py > $O/boundary_gaps.txt 2>&1 || { tail -5 $O/boundary_gaps.txt; exit 1; }
tail -4 $O/boundary_gaps.txt
