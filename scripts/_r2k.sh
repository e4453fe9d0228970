set -e
mkdir -p gpurun_out/r2k
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -q --timeout 200 --timeout-method thread -k "gemm16 or full16 or resnet50_bf16" > gpurun_out/r2k/t.txt 2>&1
for pipe in 0 1; do
  TMR_GEMM16_PIPE=$pipe timeout -k 10 200 python scripts/convbench.py --io16 --stats --bnbwd --reps 5 > gpurun_out/r2k/cb_pipe$pipe.txt 2>&1
  echo pipe=$pipe; tail -1 gpurun_out/r2k/cb_pipe$pipe.txt
done
