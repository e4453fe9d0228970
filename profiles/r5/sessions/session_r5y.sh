# experiment: trunk weight gradients on a second stream with every tensor allocated on the main
# stream (TMR_WGRAD_SIDE=1): bit-identity, then same-box C2 / C5 A/B, and a kernel trace of C2
set -o pipefail
O=gpurun_out/s5y; mkdir -p $O
timeout -k 10 300 python -u scripts/probe/side_identity.py > $O/identity.txt 2>&1 || exit 1
for rep in 1 2; do
  for s in 0 1; do
    TMR_WGRAD_SIDE=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --steps 15 > $O/c2_s${s}_$rep.json 2> $O/c2_s${s}_$rep.err || exit 1
  done
done
for s in 0 1; do
  TMR_WGRAD_SIDE=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_s$s.json 2> $O/c5_s$s.err || exit 1
done
TMR_WGRAD_SIDE=1 PROF_NAME=s5y/prof_side STEPS=3 BENCH_ARGS="--no-roofline" bash scripts/profile.sh > $O/prof.log 2>&1 || exit 1
