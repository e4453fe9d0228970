# round 5 final build (2): PMC traffic (FETCH_SIZE / WRITE_SIZE / MFMA busy) and rocprofv3 kernel stats
# of C2 fp32, C4 bf16 and C5 bf16
set -o pipefail
PROF_NAME=s5x/pmc_c2 bash scripts/pmc.sh > gpurun_out/s5x_pmc_c2.log 2>&1 || exit 1
PROF_NAME=s5x/pmc_c4 MODEL=resnest50 PRECISION=bf16 bash scripts/pmc.sh > gpurun_out/s5x_pmc_c4.log 2>&1 || exit 1
PROF_NAME=s5x/pmc_c5 PRECISION=bf16 SEQ=30 LFB=300 bash scripts/pmc.sh > gpurun_out/s5x_pmc_c5.log 2>&1 || exit 1
PROF_NAME=s5x/prof_c2 STEPS=3 bash scripts/profile.sh > gpurun_out/s5x_prof_c2.log 2>&1 || exit 1
PROF_NAME=s5x/prof_c4 STEPS=3 BENCH_ARGS="--model resnest50 --precision bf16" bash scripts/profile.sh > gpurun_out/s5x_prof_c4.log 2>&1 || exit 1
PROF_NAME=s5x/prof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh > gpurun_out/s5x_prof_c5.log 2>&1 || exit 1
