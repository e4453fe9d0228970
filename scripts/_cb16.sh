mkdir -p gpurun_out/cb16
for cfg in auto 0 1 2 3 4 5; do
  if [ $cfg = auto ]; then unset TMR_GEMM16_CFG; else export TMR_GEMM16_CFG=$cfg; fi
  timeout -k 10 150 python scripts/convbench.py --io16 --stats --bnbwd --reps 3 > gpurun_out/cb16/cfg_${cfg}.txt 2>&1 || exit 1
  echo "cfg=$cfg"; tail -1 gpurun_out/cb16/cfg_${cfg}.txt
done
