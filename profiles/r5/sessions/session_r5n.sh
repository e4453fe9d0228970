# Per-launch conv tables of the C4 / C5 / C2 steps under the old (TMR_TILE_RULE=0) and round-5
# tile rules: which launches the new rules move.
set -o pipefail
O=gpurun_out/s5n; mkdir -p $O
B="--no-cpu-baseline --conv-table"
for r in 0 1; do
  TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --model resnest50 --precision bf16 --steps 5 > $O/c4_r$r.json 2> $O/c4_r$r.err || exit 1
  TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --precision bf16 --seq 30 --lfb 300 --steps 3 > $O/c5_r$r.json 2> $O/c5_r$r.err || exit 1
  TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --steps 5 > $O/c2_r$r.json 2> $O/c2_r$r.err || exit 1
done
