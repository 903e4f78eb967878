# PMC passes for config D (bicycle 1M / 256^3, one GPU): SQ counters and
# FETCH_SIZE / WRITE_SIZE of the fused-pipeline kernels, each pass its own
# --pmc run with kernel tracing only.  -> <out>/traffic_D.json, pmc_summary_D.json
set -e
OUT=${1:-gpurun_out/pmcD}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=bicycle.json N=1000000 NG=256 NSUB=20
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$n -o run -- python3 tools/pmc_probe.py > $OUT/$n.log 2>&1
  f=$(find $OUT/$n -name run_counter_collection.csv | head -n 1); mkdir -p $OUT/$n.csv; cp "$f" $OUT/$n.csv/
  rm -rf $OUT/$n
}
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
python3 tools/traffic.py $OUT/p3.csv $OUT/p4.csv $OUT/traffic_D.json > /dev/null
python3 tools/pmc_summary.py $OUT/pmc_summary_D.json $OUT/p1.csv $OUT/p3.csv $OUT/p4.csv
echo ok
