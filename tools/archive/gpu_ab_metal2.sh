# Metal stress-path A/B: base (volume prefetched with the material planes,
# refined rsqrt behind a range branch) vs volpf0 (volume loaded after the
# return map) vs fast3 (branch-free refined rsqrt); metal parity tests on
# base and on fast3 first.
set -o pipefail
O=gpurun_out/${1:-r06m2}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_constitutive.py tests/test_gpu_parity_long.py -k "metal or constitutive or svd" > $O/tests_base.txt 2>&1 || { tail -30 $O/tests_base.txt; exit 1; }
tail -1 $O/tests_base.txt
GSMPM_LIB=$PWD/gaussian-splatting-mpm_amd/libgsmpm_fast3.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_constitutive.py tests/test_gpu_parity_long.py -k "metal or constitutive or svd" > $O/tests_fast3.txt 2>&1 || { tail -30 $O/tests_fast3.txt; }
tail -1 $O/tests_fast3.txt
VARIANTS="base volpf0 fast3" CONFIGS="C" REPS=3 bash tools/ab_libs_multi.sh $O/ab > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
