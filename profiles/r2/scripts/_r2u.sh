set -e
mkdir -p gpurun_out/r2u
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bf16_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r2u/t.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --reps 5 > gpurun_out/r2u/cb32.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --io16 --stats --bnbwd --reps 5 > gpurun_out/r2u/cb16.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2u/c2.json 2> gpurun_out/r2u/c2.err
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > gpurun_out/r2u/c2_bf16.json 2> gpurun_out/r2u/c2_bf16.err
