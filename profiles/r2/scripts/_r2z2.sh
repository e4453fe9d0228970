set -e
mkdir -p gpurun_out/r2z2
for c in 0 1 2 3 4 5 6 7; do
  TMR_GEMM16_CFG=$c timeout -k 10 200 python scripts/convbench.py --reps 4 --kinds wgrad > gpurun_out/r2z2/cfg$c.txt 2>&1
done
TMR_GEMM32=0 timeout -k 10 200 python scripts/convbench.py --reps 4 --kinds wgrad > gpurun_out/r2z2/old.txt 2>&1
