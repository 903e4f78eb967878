# The CPU suite (-m "not gpu") against the oracle's ASan + UBSan build with the
# grid-index bounds checks on (oracle/Makefile `asan`, -DOM_DEBUG).
# CPU only -- never sent to the GPU box.  Usage: bash tools/oracle_asan.sh <log>
set -o pipefail
LOG=${1:-profiles/r06/oracle_asan_cpu_suite.log}
mkdir -p "$(dirname "$LOG")"
make -s -C oracle asan || exit 1
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
{
  echo "# oracle ASan/UBSan run: $(date -u +%FT%TZ), gcc $(gcc -dumpfullversion)"
  echo "# LD_PRELOAD=$ASAN_LIB:$UBSAN_LIB GSMPM_ORACLE_VARIANT=asan ASAN_OPTIONS=detect_leaks=0:abort_on_error=1"
  LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB" GSMPM_ORACLE_VARIANT=asan \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    OMP_NUM_THREADS=4 python -m pytest tests -m "not gpu" -q -p no:cacheprovider 2>&1
} | tee "$LOG"
