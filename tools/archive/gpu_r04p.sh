# Round 4, GPU call P: does a second stream run beside the simulator's frame
# graph (tools/stream_probe.py), and the bench's host timing per call.
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 180 python3 tools/stream_probe.py > $O/stream_probe.txt 2>&1; rc=$?; cat $O/stream_probe.txt | grep -v Warning | tail -12
[ $rc -eq 0 ] || exit $rc
GSMPM_BENCH_HOST_TIMING=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 3 > $O/bench_host.json 2> $O/bench_host.err || exit 1
grep "host us" $O/bench_host.err
