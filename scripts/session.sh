# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bf16_gpu.py -k persistent -m gpu > $O/pytest_pers.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bf16_gpu.py tests/test_geometry_gpu.py tests/test_resnest_trunk_gpu.py -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 --conv-table > $O/c5.json 2> $O/c5_table.txt && \
TMR_PERSIST=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_nopers.json 2> $O/c5_nopers.err && \
TMR_FWD_SHORT_K=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_old.json 2> $O/c5_old.err && \
TMR_FWD_SHORT_CFG=7 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_cfg7.json 2> $O/c5_cfg7.err && \
TMR_RELU_BITS16=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_bits.json 2> $O/c5_bits.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 --conv-table > $O/c4.json 2> $O/c4_table.txt && \
TMR_FWD_SHORT_K=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4_old.json 2> $O/c4_old.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --conv-table > $O/c2.json 2> $O/c2_table.txt && \
TMR_FWD_SHORT_K=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2_old.json 2> $O/c2_old.err
echo "main rc=$?"
