set -e
OUT=gpurun_out/pmcD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CONFIG=bicycle.json N=1000000 NG=256 NSUB=10
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o run -- python3 tools/pmc_probe.py > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/p2 -o run -- python3 tools/pmc_probe.py > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- python3 tools/pmc_probe.py > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- python3 tools/pmc_probe.py > $OUT/p4.log 2>&1
python3 tools/traffic.py $OUT/p3 $OUT/p4 $OUT/traffic.json > /dev/null
echo ok
