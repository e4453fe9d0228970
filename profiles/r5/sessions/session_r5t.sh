# split-attention reductions with 4 pixels in flight: ResNeSt tests, then a same-box C4 A/B against the
# previous build (libtmr_ab.so), interleaved
set -o pipefail
O=gpurun_out/s5t; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_resnest_gpu.py -k "avgpool or splat or resnest" > $O/pytest.txt 2>&1 || exit 1
B="--no-cpu-baseline --model resnest50 --precision bf16 --steps 10"
for rep in 1 2; do
  TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_ab.so timeout -k 10 200 python -u bench.py $B > $O/c4_old_$rep.json 2> $O/c4_old_$rep.err || exit 1
  timeout -k 10 200 python -u bench.py $B > $O/c4_new_$rep.json 2> $O/c4_new_$rep.err || exit 1
done
PROF_NAME=s5t/prof_c4 STEPS=3 BENCH_ARGS="--model resnest50 --precision bf16" bash scripts/profile.sh > $O/prof_c4.log 2>&1 || exit 1
