# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
PROF_NAME=r5u/rocprof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh > $O/prof_c5.txt 2>&1 && \
PROF_NAME=r5u/rocprof_c4 STEPS=8 BENCH_ARGS="--model resnest50 --precision bf16" bash scripts/profile.sh > $O/prof_c4.txt 2>&1
echo "main rc=$?"
