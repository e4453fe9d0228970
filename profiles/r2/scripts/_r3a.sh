set -e
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a/t_kernels.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3a/pytest_gpu.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3a/bench_fp32.json 2> gpurun_out/r3a/bench_fp32.err
TMR_RELU_BITS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3a/bench_fp32_nobits.json 2> gpurun_out/r3a/bench_fp32_nobits.err
