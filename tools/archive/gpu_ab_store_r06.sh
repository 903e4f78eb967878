# Store policies after the XCD grouping: window slots plain (sl0) / nt (sl1)
# instead of write-through, v_out write-through (gv2) / nt (gv1) instead of
# plain; 3 interleaved rounds on B and C, 2 on B'.
set -o pipefail
O=gpurun_out/${1:-r06st}; mkdir -p $O
VARIANTS="base sl0 sl1 gv2 gv1" CONFIGS="B C" REPS=3 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
