# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && TMR_LSTM_PERSIST=0 timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/probe_lstm_steps -o run -- python3 $R/scripts/exit_probe.py lstm > $R/$O/probe_lstm_steps.log 2>&1 ) && echo "probe lstm per-step rc=0" && \
PROF_NAME=r4g/prof_c2 STEPS=3 bash scripts/profile.sh && \
PROF_NAME=r4g/prof_c4 STEPS=3 BENCH_ARGS="--model resnest50 --precision bf16" bash scripts/profile.sh && \
PROF_NAME=r4g/prof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh && \
PROF_NAME=r4g/pmc_c2 bash scripts/pmc.sh && \
PROF_NAME=r4g/pmc_c4 MODEL=resnest50 PRECISION=bf16 bash scripts/pmc.sh
echo "main rc=$?"
