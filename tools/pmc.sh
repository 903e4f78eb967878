# PMC passes for the lego frame kernels (run on the GPU box via gpurun).
# Each counter group is its own --pmc run with kernel tracing only (no
# sys/runtime trace); FETCH_SIZE and WRITE_SIZE each get a pass of their own.
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export RENDER=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$n -o run -- python3 tools/pmc_probe.py > $OUT/$n.log 2>&1
  f=$(find $OUT/$n -name run_counter_collection.csv | head -n 1); mkdir -p $OUT/$n.csv; cp "$f" $OUT/$n.csv/
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
run p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS
run p3 FETCH_SIZE
run p4 WRITE_SIZE
python3 tools/traffic.py $OUT/p3.csv $OUT/p4.csv $OUT/traffic.json > /dev/null
python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/p1.csv $OUT/p2.csv $OUT/p3.csv $OUT/p4.csv
echo ok
