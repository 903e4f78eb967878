# PMC passes of the bicycle render alone (tools/render_probe.py, CONFIG=bicycle):
# SQ counters and FETCH/WRITE of k_emit_pairs, k_render, k_preprocess, sorts.
set -e
O=${1:-gpurun_out/pmc_render_D}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=bicycle.json N=1000000 NG=256 REPS=3
run() {
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/$n -o run -- python3 tools/render_probe.py > $O/$n.log 2>&1
  f=$(find $O/$n -name run_counter_collection.csv | head -n 1); mkdir -p $O/$n.csv; cp "$f" $O/$n.csv/
  rm -rf $O/$n
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY
run p3 FETCH_SIZE
run p4 WRITE_SIZE
python3 tools/pmc_summary.py $O/pmc_summary.json $O/p1.csv $O/p3.csv $O/p4.csv
echo ok
