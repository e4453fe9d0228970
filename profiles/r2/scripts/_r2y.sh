set -e
mkdir -p gpurun_out/r2y
for c in 0 1 2 3 4 5 6 7; do
  TMR_GEMM16_CFG=$c timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --wt32 --reps 4 --kinds fwd,dgrad > gpurun_out/r2y/cfg$c.txt 2>&1
done
