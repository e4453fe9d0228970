set -e
mkdir -p gpurun_out/r2z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2z/pytest_gpu.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2z/bench_fp32.json 2> gpurun_out/r2z/bench_fp32.err
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > gpurun_out/r2z/c2_bf16.json 2> gpurun_out/r2z/c2_bf16.err
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --model resnest50 > gpurun_out/r2z/c4_bf16.json 2> gpurun_out/r2z/c4_bf16.err
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2z/c5_bf16.json 2> gpurun_out/r2z/c5_bf16.err
