set -e
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b/t_kernels.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --wt32 --reps 5 --kinds dgrad --dgrad-beta 1 > gpurun_out/r3b/cb32_dgrad.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --io16 --stats --bnbwd --reps 5 --kinds dgrad --dgrad-beta 1 > gpurun_out/r3b/cb16_dgrad.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3b/bench_fp32.json 2> gpurun_out/r3b/bench_fp32.err
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > gpurun_out/r3b/c2_bf16.json 2> gpurun_out/r3b/c2_bf16.err
