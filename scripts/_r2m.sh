set -e
PROF_NAME=r2m/prof_bf16 STEPS=5 BENCH_ARGS="--precision bf16" bash scripts/profile.sh
PROF_NAME=r2m/pmc_bf16 PRECISION=bf16 bash scripts/pmc.sh
