set -e
mkdir -p gpurun_out/r2v
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bf16_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r2v/t.txt 2>&1
timeout -k 10 200 python scripts/convbench.py --io16 --stats --bnbwd --reps 5 > gpurun_out/r2v/cb16.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > gpurun_out/r2v/c2_bf16.json 2> gpurun_out/r2v/c2_bf16.err
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2v/c5_bf16.json 2> gpurun_out/r2v/c5_bf16.err
PROF_NAME=r2v/pmc PRECISION=bf16 bash scripts/pmc.sh > gpurun_out/r2v/pmc.log 2>&1
