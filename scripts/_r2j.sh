set -e
mkdir -p gpurun_out/r2j
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_geometry_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2j/bf16t.txt 2>&1 || true
timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2j/c2_bf16.json 2> gpurun_out/r2j/c2_bf16.err
TMR_BF16_ACT=0 timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2j/c2_bf16_act32.json 2> gpurun_out/r2j/c2_bf16_act32.err
timeout -k 10 300 python bench.py $B --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2j/c5_bf16.json 2> gpurun_out/r2j/c5_bf16.err
