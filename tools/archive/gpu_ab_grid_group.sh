# XCD-grouped k_grid_f work order (GSMPM_GRID_GROUP): the fused/config/slab
# tests on the new default (16), an interleaved A/B against 4 and the plain
# order (grp0) on B, B' and D, and FETCH_SIZE / WRITE_SIZE for base and grp0
# on config B.
set -o pipefail
O=gpurun_out/${1:-r06grp}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mpm.py tests/test_gpu_configs.py tests/test_gpu_slab.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
VARIANTS="base grp4 grp0" CONFIGS="B Bp D" REPS=2 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=lego.json N=100000 NG=128 NSUB=20
for v in base grp0; do
  if [ $v = grp0 ]; then export GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_grp0.so; else unset GSMPM_LIB; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python3 tools/pmc_probe.py > $O/pmc_${v}_$c.log 2>&1 || exit 1
    mkdir -p $O/d_${v}_$c; f=$(find $O/pmc_${v}_$c -name run_counter_collection.csv | head -n 1); cp "$f" $O/d_${v}_$c/; rm -rf $O/pmc_${v}_$c
  done
  python3 tools/traffic.py $O/d_${v}_FETCH_SIZE $O/d_${v}_WRITE_SIZE $O/traffic_$v.json > /dev/null
  python3 -c "import json; d=json.load(open('$O/traffic_$v.json'))['kernels']; print('$v', {k: (round(d[k]['fetch_bytes']/1e6,2), round(d[k]['write_bytes']/1e6,2)) for k in ('k_fused','k_grid_f')})"
done
