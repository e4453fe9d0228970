set -o pipefail
O=gpurun_out/s5g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_modules_gpu.py tests/test_compat_gpu.py > $O/pytest_lstm.txt 2>&1 || exit 1
B="timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --conv-table"
for k in 0 64 128 256; do
  TMR_NST1_K32=$k $B > $O/c2_k$k.json 2> $O/c2_k$k.err || exit 1
done
TMR_NST1_K32=0 $B > $O/c2_k0b.json 2> $O/c2_k0b.err || exit 1
# the persistent LSTM (plain launch) under rocprofv3: does the process exit 0 now?
PROF_NAME=s5g/prof_persist TMR_LSTM_PERSIST=1 STEPS=3 bash scripts/profile.sh > $O/prof_persist.log 2>&1
echo "profile rc=$?" >> $O/prof_persist.log
