# strided dgrads: tile order of the one-launch form (chunks of G tiles per class) vs per-class launches
set -o pipefail
R=$PWD
O=$R/gpurun_out/s5aj; mkdir -p $O
S=128:128:3:56,256:256:3:28,512:512:3:14,256:512:1:56,512:1024:1:28,1024:2048:1:14
for m in cl g32 g64 g128 g256; do
  F=""; E="TMR_PAR_ORDER=2 TMR_PAR_G=${m#g}"
  [ $m = cl ] && F="--classes" && E="TMR_PAR_ORDER=0"
  timeout -k 10 200 env $E python scripts/convbench.py --frames 1920 --reps 5 --io16 --bnbwd --kinds dgrad --only $S $F > $O/bf16_$m.log 2>&1 || exit 1
  timeout -k 10 200 env $E python scripts/convbench.py --frames 640 --reps 5 --wt32 --bnbwd --kinds dgrad --only $S $F > $O/f32_$m.log 2>&1 || exit 1
done
