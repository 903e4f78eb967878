# PMC passes for another BASELINE configuration on one GPU (CONFIG, N, NG,
# MAT in the environment, as tools/pmc_probe.py reads them): FETCH_SIZE /
# WRITE_SIZE and the SQ counters of the fused-pipeline kernels, each pass its
# own --pmc run with kernel tracing only.
# usage: CONFIG=... N=... NG=... MAT=... bash tools/pmc_cfg.sh <out> <tag>
#   -> <out>/traffic_<tag>.json, <out>/pmc_summary_<tag>.json
set -e
OUT=${1:-gpurun_out/pmc_cfg}
TAG=${2:-cfg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export NSUB=${NSUB:-20}
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$n -o run -- python3 tools/pmc_probe.py > $OUT/$n.log 2>&1
  f=$(find $OUT/$n -name run_counter_collection.csv | head -n 1); mkdir -p $OUT/$n.csv; cp "$f" $OUT/$n.csv/
  rm -rf $OUT/$n
}
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
python3 tools/traffic.py $OUT/p3.csv $OUT/p4.csv $OUT/traffic_$TAG.json > /dev/null
python3 tools/pmc_summary.py $OUT/pmc_summary_$TAG.json $OUT/p1.csv $OUT/p3.csv $OUT/p4.csv
echo ok
