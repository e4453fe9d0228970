# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bf16_gpu.py -k "g16 or fused_bn" -m gpu > $O/pytest_g16.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || exit $?
for c in 7 5; do
  TMR_DGRAD32_WIDE_CFG=$c timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --conv-table > $O/c2_w$c.json 2> $O/c2_w${c}_table.txt || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 --conv-table > $O/c5.json 2> $O/c5_table.txt && \
TMR_G16=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_nog16.json 2> $O/c5_nog16.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4.json 2> $O/c4.err
echo "main rc=$?"
