# Tile-config sweep of the current engine (round 5 epilogues): every conv view of the C2 (fp32,
# 640 frames) and C5 (bf16, 1920 frames) train steps with each tile config forced, against auto.
# A Python error (a config the launcher rejects) moves on; a timeout / signal ends the session.
set -o pipefail
O=gpurun_out/s5l; mkdir -p $O
run() {  # name, env / command ...
  local n=$1; shift
  timeout -k 10 150 env "$@" > $O/$n.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAIL $n rc=$rc"; tail -3 $O/$n.log; [ $rc -eq 1 ] || exit $rc; fi
  tail -1 $O/$n.log
}
for c in auto 1 2 3 5 6 7; do
  E=""; [ $c != auto ] && E="TMR_GEMM16_CFG=$c"
  run f32_$c $E python scripts/convbench.py --frames 640 --reps 5 --wt32 --stats --bnbwd --json $O/f32_$c.json
done
for c in auto 1 2 3 5 6 7; do
  E=""; [ $c != auto ] && E="TMR_GEMM16_CFG=$c"
  run b16_$c $E python scripts/convbench.py --frames 1920 --reps 3 --io16 --stats --y16 --bnbwd --json $O/b16_$c.json
done
