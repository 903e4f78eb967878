# Round 4, GPU call M: (1) the render alone on the default stream vs a second
# stream, wall and event timing (the bench breakdown reads ~0.25 ms against
# the probe's ~0.16); (2) the s_setprio variant of the simulator kernels on the
# lego bench frame (3 interleaved rounds).
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
for i in 1 2; do for rs in 0 1; do for ev in 0 1; do
  echo "rstream=$rs events=$ev $(RSTREAM=$rs EVENTS=$ev REPS=50 timeout -k 10 120 python3 tools/render_probe.py 2>&1 | tail -n 1)"
done; done; done | tee $O/render_stream.txt
REPS=3 bash tools/ab_libs.sh base prio > $O/ab_prio.txt 2>&1 || exit 1
cat $O/ab_prio.txt
