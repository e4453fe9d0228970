set -o pipefail
O=gpurun_out/s5k; mkdir -p $O
PROF_NAME=s5k/prof_side TMR_WGRAD_STREAM=1 STEPS=3 bash scripts/profile.sh > $O/prof_side.log 2>&1 || exit 1
