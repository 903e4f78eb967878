# A/B of two builds of libgsmpm on the render alone (tools/render_probe.py):
# bicycle (1M / 256^3) and lego, 3 interleaved pairs, then a rocprofv3
# kernel-stats pass of each build on the bicycle.
#   bash tools/ab_render_lib.sh <libA.so> <libB.so> <out>
set -e
A=$1; B=$2; O=${3:-gpurun_out/ab_render_lib}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for L in A B; do
    if [ $L = A ]; then LIB=$A; else LIB=$B; fi
    GSMPM_LIB=$LIB CONFIG=bicycle.json N=1000000 NG=256 REPS=10 timeout -k 10 240 python3 tools/render_probe.py > $O/bicycle.$L.$i.log 2>&1
    echo "bicycle $L $(tail -n 1 $O/bicycle.$L.$i.log)"
    GSMPM_LIB=$LIB REPS=50 timeout -k 10 120 python3 tools/render_probe.py > $O/lego.$L.$i.log 2>&1
    echo "lego $L $(tail -n 1 $O/lego.$L.$i.log)"
  done
done
for L in A B; do
  if [ $L = A ]; then LIB=$A; else LIB=$B; fi
  GSMPM_LIB=$LIB CONFIG=bicycle.json N=1000000 NG=256 REPS=5 timeout -k 10 240 \
    rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$L -o run -- python3 tools/render_probe.py > $O/prof$L.log 2>&1
  f=$(find $O/prof$L -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/bicycle_kernel_stats_$L.csv
done
echo ok
