# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4_new$i.json 2> $O/c4_new$i.err || exit $?
TMR_LIB_PATH=tmrnet_amd/libtmr_prev.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4_prev$i.json 2> $O/c4_prev$i.err || exit $?
done
echo "main rc=$?"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_kernels_gpu.py tests/test_geometry_gpu.py -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --precision bf16 --seq 30 --lfb 300 > $O/c5.json 2> $O/c5.err
echo "tail rc=$?"
