set -e
mkdir -p gpurun_out/r2o
B="--no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 500 python -u -m pytest tests/test_bf16_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2o/t.txt 2>&1 || true
timeout -k 10 200 python scripts/convbench.py --io16 --kinds dgrad --bnbwd --reps 5 > gpurun_out/r2o/cb_dgrad.txt 2>&1
timeout -k 10 200 python bench.py $B --precision bf16 > gpurun_out/r2o/c2_bf16.json 2> gpurun_out/r2o/c2_bf16.err
