mkdir -p gpurun_out/cb32
timeout -k 10 200 python scripts/convbench.py --stats --bnbwd --reps 5 > gpurun_out/cb32/auto.txt 2>&1
