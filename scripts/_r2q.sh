set -e
mkdir -p gpurun_out/r2q
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -q --timeout 200 --timeout-method thread -k "gemm16 or full16 or resnet50_bf16" > gpurun_out/r2q/t.txt 2>&1 || true
timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2q/c2_bf16.json 2> gpurun_out/r2q/c2_bf16.err
timeout -k 10 300 python bench.py $B --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2q/c5_bf16.json 2> gpurun_out/r2q/c5_bf16.err
timeout -k 10 300 python bench.py $B --precision bf16 --model resnest50 > gpurun_out/r2q/c4_bf16.json 2> gpurun_out/r2q/c4_bf16.err
