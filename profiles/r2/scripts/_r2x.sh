set -e
mkdir -p gpurun_out/r2x
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2x/t_kernels.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --wt32 --reps 5 > gpurun_out/r2x/cb32_dma.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2x/pytest_gpu.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2x/bench_fp32.json 2> gpurun_out/r2x/bench_fp32.err
