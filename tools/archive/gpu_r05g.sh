# Round 5, GPU call G: the MPM + raster GPU tests with the wave-aggregated
# re-binning slots, k_fused LDS conflicts per build (PMC), the bench A/B of
# the aggregation, k_grid_f's per-workgroup phases with / without the cover
# records (stamps build), the render CU-mask layouts, and the two-rank
# rehearsal line (both ranks on this GPU).
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mpm.py tests/test_gpu_raster.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -15; [ $rc = 0 ] || exit 1
bash tools/lds_conflicts.sh $O/lds "agg||" "lane|binlane|" "agg_nolb||GSMPM_LANE_BALANCE=0" || exit 1
REPS=3 bash tools/ab_r05.sh $O/ab "agg||" "lane|binlane|" || exit 1
for rec in 1 0; do
  GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_stamps.so GSMPM_COVER_RECORDS=$rec TAG=records$rec \
    timeout -k 10 150 python3 tools/grid_f_phases.py >> $O/grid_f_phases.txt 2> $O/phases_$rec.err || { tail -5 $O/phases_$rec.err; exit 1; }
done
cat $O/grid_f_phases.txt
REPS=2 bash tools/ab_r05.sh $O/cus "thread||" "spread16||GSMPM_BENCH_RENDER_CUS=16" \
  "low16||GSMPM_BENCH_RENDER_CUS=16 GSMPM_BENCH_RENDER_CU_LAYOUT=low" "xmajor16||GSMPM_BENCH_RENDER_CUS=16 GSMPM_BENCH_RENDER_CU_LAYOUT=xmajor" \
  "low8||GSMPM_BENCH_RENDER_CUS=8 GSMPM_BENCH_RENDER_CU_LAYOUT=low" "xmajor8||GSMPM_BENCH_RENDER_CUS=8 GSMPM_BENCH_RENDER_CU_LAYOUT=xmajor" || exit 1
GSMPM_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 --multi-configs lego,split \
  > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err || { tail -20 $O/rehearsal_2ranks.err; exit 1; }
tail -1 $O/rehearsal_2ranks.json | cut -c1-1500
