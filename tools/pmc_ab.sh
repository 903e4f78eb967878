# LDS counters of the lego frame kernels with an env toggle on / off (GPU box):
#   bash tools/pmc_ab.sh VAR "v1 v2"
set -e
VAR=$1; VALS=$2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $VALS; do
  O=gpurun_out/pmcab_$v
  mkdir -p $O
  env $VAR=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 tools/pmc_probe.py > $O/p1.log 2>&1
  f=$(find $O/p1 -name run_counter_collection.csv | head -n 1); mkdir -p $O/p1.csv; cp "$f" $O/p1.csv/; rm -rf $O/p1
  python3 tools/pmc_summary.py $O/summary.json $O/p1.csv
  python3 -c "
import json; d=json.load(open('$O/summary.json'))['per_dispatch_average']
for k,v in d.items():
    if 'k_fused' in k or 'k_grid_f' in k: print('$VAR=$v', k, {c: round(x) if isinstance(x,float) and x>10 else x for c,x in v.items()})"
done
