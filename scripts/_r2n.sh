set -e
mkdir -p gpurun_out/r2n
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 500 python -u -m pytest tests/test_resnest_gpu.py tests/test_bf16_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2n/t.txt 2>&1 || true
timeout -k 10 300 python bench.py $B --precision bf16 --model resnest50 > gpurun_out/r2n/c4_bf16.json 2> gpurun_out/r2n/c4_bf16.err
TMR_BF16_FULL=0 timeout -k 10 300 python bench.py $B --precision bf16 --model resnest50 > gpurun_out/r2n/c4_bf16_old.json 2> gpurun_out/r2n/c4_bf16_old.err
