# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_geometry_gpu.py tests/test_kernels_gpu.py -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5.json 2> $O/c5.err && \
TMR_BN8=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5_bn4.json 2> $O/c5_bn4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4.json 2> $O/c4.err && \
TMR_BN8=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4_bn4.json 2> $O/c4_bn4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2.json 2> $O/c2.err
echo "main rc=$?"
