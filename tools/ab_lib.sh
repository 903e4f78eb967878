# A/B of two builds of libgsmpm on one box (render and frame times from
# bench.py, 3 interleaved pairs): bash tools/ab_lib.sh <libA.so> <libB.so> <out>
set -e
A=$1; B=$2; O=${3:-gpurun_out/ab_lib}
mkdir -p $O
for i in 1 2 3; do
  for L in A B; do
    if [ $L = A ]; then LIB=$A; else LIB=$B; fi
    GSMPM_LIB=$LIB timeout -k 10 120 python3 bench.py --no-extra-configs --no-cpu-baseline --steps 10 --warmup 3 > $O/$L.$i.log 2>&1
    python3 -c "import json; d=json.loads(open('$O/$L.$i.log').read().strip().splitlines()[-1]); print('$L', round(d['render_ms_per_frame'],4), 'ms render;', round(d['sim_ms_per_frame'],4), 'ms sim;', round(d['ms_per_step'],4), 'ms frame;', '%.4g' % d['value'])"
  done
done
