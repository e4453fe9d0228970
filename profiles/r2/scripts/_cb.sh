cd $GRAFT_REPO_ROOT
for cfg in auto 4 0 5 7 8; do
  if [ $cfg = auto ]; then unset TMR_GEMM_CFG; else export TMR_GEMM_CFG=$cfg; fi
  timeout -k 10 150 python scripts/convbench.py --math bf16 --stats --reps 3 > gpurun_out/cbb_${cfg}.txt 2>&1 || exit 1
  echo "cfg=$cfg"; tail -1 gpurun_out/cbb_${cfg}.txt
done
