set -e
mkdir -p gpurun_out/r2e
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e/pytest_gpu.txt 2>&1
timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2e/c2_bf16.json 2> gpurun_out/r2e/c2_bf16.err
TMR_BF16_STORE=0 timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2e/c2_bf16_nostore.json 2> gpurun_out/r2e/c2_bf16_nostore.err
timeout -k 10 300 python bench.py $B --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2e/c5_bf16.json 2> gpurun_out/r2e/c5_bf16.err
TMR_BF16_STORE=0 timeout -k 10 300 python bench.py $B --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2e/c5_bf16_nostore.json 2> gpurun_out/r2e/c5_bf16_nostore.err
timeout -k 10 300 python bench.py $B --precision bf16 --model resnest50 > gpurun_out/r2e/c4_bf16.json 2> gpurun_out/r2e/c4_bf16.err
timeout -k 10 300 python bench.py $B > gpurun_out/r2e/c2_fp32.json 2> gpurun_out/r2e/c2_fp32.err
