# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
PROF_NAME=r5t/pmc bash scripts/pmc.sh > $O/pmc.txt 2>&1 && \
PROF_NAME=r5t/rocprof_c2 STEPS=8 bash scripts/profile.sh > $O/prof_c2.txt 2>&1
echo "main rc=$?"
