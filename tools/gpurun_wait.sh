# gpurun, re-queued only while the pod has no free GPU slot (exit 3: nothing ran,
# nothing charged); any other outcome -- success or failure -- is final.
# usage: bash tools/gpurun_wait.sh <timeout-s> '<command>'
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
