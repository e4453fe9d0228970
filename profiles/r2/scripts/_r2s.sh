set -e
mkdir -p gpurun_out/r2s
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 500 python -u -m pytest tests/test_bf16_gpu.py tests/test_resnest_gpu.py tests/test_geometry_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2s/t.txt 2>&1 || true
timeout -k 10 200 python scripts/convbench.py --io16 --stats --bnbwd --reps 5 > gpurun_out/r2s/cb.txt 2>&1
timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2s/c2_bf16.json 2> gpurun_out/r2s/c2_bf16.err
timeout -k 10 300 python bench.py $B --precision bf16 --seq 30 --lfb 300 > gpurun_out/r2s/c5_bf16.json 2> gpurun_out/r2s/c5_bf16.err
timeout -k 10 300 python bench.py $B --precision bf16 --model resnest50 > gpurun_out/r2s/c4_bf16.json 2> gpurun_out/r2s/c4_bf16.err
