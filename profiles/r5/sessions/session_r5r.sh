# experiment: stagger the second workgroup slot of each CU in the fused BN-backward dgrads
set -o pipefail
O=gpurun_out/s5r; mkdir -p $O
for s in 0 1 2 3 5 0; do
  TMR_STAGGER=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --conv-table > $O/c2_s$s.json 2> $O/c2_s$s.err || exit 1
done
for s in 0 2; do
  TMR_STAGGER=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 --steps 5 --conv-table > $O/c5_s$s.json 2> $O/c5_s$s.err || exit 1
done
