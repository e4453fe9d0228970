# experiment: 256x256 as 4 waves (128x128 per wave, cfg 8) on the bf16 forwards / wgrads at C5 size
set -o pipefail
O=gpurun_out/s5ah; mkdir -p $O
for c in 8; do
  E=""; [ $c != auto ] && E="TMR_GEMM16_CFG=$c"
  timeout -k 10 200 env $E python scripts/convbench.py --frames 1920 --reps 3 --io16 --stats --y16 --kinds fwd,wgrad --only 64:256:1:56,128:512:1:28,256:1024:1:14,512:2048:1:7,256:256:3:14,512:512:3:7,128:128:3:28,1024:256:1:14,512:128:1:28 > $O/cfg_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
