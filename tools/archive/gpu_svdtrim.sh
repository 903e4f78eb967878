# SVD trim (GSMPM_SVD_TRIM): the constitutive / metal parity tests on the new
# default build, then an interleaved metal + lego A/B against the plain form.
set -o pipefail
O=gpurun_out/${1:-r06svd}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_constitutive.py tests/test_gpu_parity_long.py tests/test_gpu_configs.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
VARIANTS="base trim0" CONFIGS="C B" REPS=3 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
