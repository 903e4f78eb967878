# k_fused's LDS bank conflicts per library build / switch (GPU box): one
# rocprofv3 --pmc pass (8 SQ counters, kernel tracing only) of the eager lego
# frame (tools/pmc_probe.py) per spec, summarized per kernel.
# usage: bash tools/lds_conflicts.sh OUT "name|lib|ENV=.. ENV2=.." ...
set -o pipefail
O=$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  IFS='|' read -r name lib envs <<< "$spec"
  if [ -z "$lib" ]; then L=$PWD/gaussian-splatting-mpm_amd/libgsmpm.so; else L=$PWD/gaussian-splatting-mpm_amd/libgsmpm_$lib.so; fi
  ( export GSMPM_LIB=$L; for e in $envs; do export "$e"; done
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
      SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/$name -o run -- python3 tools/pmc_probe.py \
      > $O/$name.log 2>&1 ) || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  f=$(find $O/$name -name run_counter_collection.csv | head -n 1)
  mkdir -p $O/$name.csv && cp "$f" $O/$name.csv/ && rm -rf $O/$name
  python3 tools/pmc_summary.py $O/$name.json $O/$name.csv > /dev/null || exit 1
  python3 - "$O/$name.json" "$name" <<'PY' | tee -a $O/summary.txt
import json, sys
d = json.load(open(sys.argv[1]))["per_dispatch_average"]
for k in ("k_fused<0, 3>", "k_fused<0, 2>", "k_fused<0, 1>"):
    v = d.get(k)
    if v:
        print(sys.argv[2], k, "conflict/active %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)),
              "lds wait/wave cycles %.4f" % (v["SQ_WAIT_INST_LDS"] / max(v["SQ_WAVE_CYCLES"], 1)),
              "LDS insts/wave %.1f" % (v["SQ_INSTS_LDS"] / max(v["SQ_WAVES"], 1)),
              "VALU insts/wave %.1f" % (v["SQ_INSTS_VALU"] / max(v["SQ_WAVES"], 1)),
              "conflict %.0f active %.0f dispatches %d" % (v["SQ_LDS_BANK_CONFLICT"], v["SQ_LDS_IDX_ACTIVE"], v["dispatches"]))
PY
done
echo ok
