# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: the wave-specialised persistent dgrad, whole-step A/B (TMR_DGRAD_WS=0: the one-tile
# launches), interleaved on one box
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_ws_a.json 2> $O/c2_ws_a.err || exit 1
TMR_DGRAD_WS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_tiles_a.json 2> $O/c2_tiles_a.err || exit 2
timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5_ws_a.json 2> $O/c5_ws_a.err || exit 3
TMR_DGRAD_WS=0 timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5_tiles_a.json 2> $O/c5_tiles_a.err || exit 4
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_ws_b.json 2> $O/c2_ws_b.err || exit 5
TMR_DGRAD_WS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_tiles_b.json 2> $O/c2_tiles_b.err || exit 6
python - <<'PY'
import json
for w in ('c2_ws_a','c2_tiles_a','c5_ws_a','c5_tiles_a','c2_ws_b','c2_tiles_b'):
    d=json.load(open('gpurun_out/r6m/%s.json'%w))
    print(w, d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
