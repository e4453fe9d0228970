# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
PROF_NAME=r5i/rocprof_c2 STEPS=3 bash scripts/profile.sh > gpurun_out/r5i_c2.log 2>&1 || exit $?
PROF_NAME=r5i/rocprof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh > gpurun_out/r5i_c5.log 2>&1 || exit $?
PROF_NAME=r5i/rocprof_c4 STEPS=3 BENCH_ARGS="--model resnest50 --precision bf16" bash scripts/profile.sh > gpurun_out/r5i_c4.log 2>&1 || exit $?
PROF_NAME=r5i/pmc_c2 bash scripts/pmc.sh > gpurun_out/r5i_pmc_c2.log 2>&1 || exit $?
echo "main rc=$?"
