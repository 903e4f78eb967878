# Round 5, GPU call AO: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1)
# against the default, interleaved on the lego bench: does the kernarg
# fetch sit in the ~1.7 us kernel-boundary gaps of the replayed graphs?
set -o pipefail
O=gpurun_out/r05ao
mkdir -p $O
REPS=4 bash tools/ab_r05.sh $O/ab "def||" "devka||HIP_FORCE_DEV_KERNARG=1" || exit 1
