set -e
mkdir -p gpurun_out/r3j
for c in 1 2 3 5 7; do
  TMR_GEMM16_CFG=$c timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --wt32 --dgrad-beta 1 --reps 4 --kinds dgrad > gpurun_out/r3j/cfg$c.txt 2>&1
done
