# Owner-grouped window slots (GSMPM_OWNER_SLOTS=1, libgsmpm_own1.so) re-measured
# on the round-6 kernels: fused/config tests on the variant, an interleaved
# A/B on B, B' and D, and FETCH_SIZE / WRITE_SIZE passes for both on config B.
set -o pipefail
O=gpurun_out/${1:-r06own}; mkdir -p $O
L1=$PWD/gaussian-splatting-mpm_amd/libgsmpm_own1.so
GSMPM_LIB=$L1 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mpm.py tests/test_gpu_configs.py -k "not bicycle and not D_" > $O/tests_own1.txt 2>&1 || { tail -30 $O/tests_own1.txt; exit 1; }
tail -1 $O/tests_own1.txt
VARIANTS="base own1" CONFIGS="B Bp D" REPS=2 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=lego.json N=100000 NG=128 NSUB=20
for v in base own1; do
  if [ $v = own1 ]; then export GSMPM_LIB=$L1; else unset GSMPM_LIB; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python3 tools/pmc_probe.py > $O/pmc_${v}_$c.log 2>&1 || exit 1
    f=$(find $O/pmc_${v}_$c -name run_counter_collection.csv | head -n 1); cp "$f" $O/${v}_$c.csv; rm -rf $O/pmc_${v}_$c
  done
  python3 tools/traffic.py $O/${v}_FETCH_SIZE.csv $O/${v}_WRITE_SIZE.csv $O/traffic_$v.json > $O/traffic_$v.txt
  echo $v; grep -i -E "k_grid_f|k_fused" $O/traffic_$v.txt | head -6
done
