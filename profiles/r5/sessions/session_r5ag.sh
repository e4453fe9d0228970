# fp32 56x56 64-channel convs (C2 layer1): every tile config forced, all three views
set -o pipefail
O=gpurun_out/s5ag; mkdir -p $O
for c in auto 0 1 2 3 4 5 6 7; do
  E=""; [ $c != auto ] && E="TMR_GEMM16_CFG=$c"
  timeout -k 10 120 env $E python scripts/convbench.py --frames 640 --reps 10 --wt32 --stats --bnbwd --only 64:64:3:56,64:64:1:56,64:256:1:56,256:64:1:56 > $O/cfg_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
