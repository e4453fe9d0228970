# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bf16_gpu.py -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 --conv-table > $O/c5.json 2> $O/c5_table.txt && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 --conv-table > $O/c4.json 2> $O/c4_table.txt && \
timeout -k 10 300 python bench.py --no-cpu-baseline --conv-table > $O/c2.json 2> $O/c2_table.txt && \
timeout -k 10 400 python scripts/decode_bench.py --workers 8,16 > $O/decode.jsonl 2> $O/decode.err
echo "main rc=$?"
