# fp32 stem on the 8-channel maxpool forward and the per-quad backward apply: stem tests, then a
# same-box C2 A/B against the previous build (libtmr_ab.so), interleaved, twice; C2 kernel stats
set -o pipefail
O=gpurun_out/s5aa; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_stem_pool8_gpu.py tests/test_kernels_gpu.py -k "stem or pool or maxpool" > $O/pytest.txt 2>&1 || exit 1
B="--no-cpu-baseline --no-roofline --steps 15"
for rep in 1 2; do
  TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_ab.so timeout -k 10 200 python -u bench.py $B > $O/c2_old_$rep.json 2> $O/c2_old_$rep.err || exit 1
  timeout -k 10 200 python -u bench.py $B > $O/c2_new_$rep.json 2> $O/c2_new_$rep.err || exit 1
done
PROF_NAME=s5aa/prof_c2 STEPS=3 bash scripts/profile.sh > $O/prof_c2.log 2>&1 || exit 1
