# Round 5, GPU call AG: does the overlapped render share a hardware queue with
# the simulator's graphs?  The frame's render tax grew with the graph segment
# length (call AF: rebin 20 / 25 / 50 -> frame - sim 0.22 / 0.38 / 1.03 ms),
# as if the render's kernels ran only between segments.  HIP maps streams
# onto GPU_MAX_HW_QUEUES hardware queues (4 on the box; torch's stream pool
# alone creates 32 streams): the lego bench at 4 (default), 8 and 16 queues,
# interleaved, and at 16 with --rebin 50.
set -o pipefail
O=gpurun_out/r05ag
mkdir -p $O
REPS=3 bash tools/ab_r05.sh $O/ab "q4||" "q8||GPU_MAX_HW_QUEUES=8" "q16||GPU_MAX_HW_QUEUES=16" || exit 1
REPS=1 BENCH_ARGS="--rebin 50" bash tools/ab_r05.sh $O/ab_r50 "q4||" "q16||GPU_MAX_HW_QUEUES=16" || exit 1
