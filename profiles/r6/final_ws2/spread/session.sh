# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6 final build (wave-specialised dgrad): the bench lines reading this build's PMC records
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/c2_1.json 2> $O/c2_1.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/c2_2.json 2> $O/c2_2.err || exit 2
timeout -k 10 300 python -u bench.py --model resnest50 --precision bf16 --steps 10 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 3
timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 4
python - <<'PY'
import json
for w in ('c2_1','c2_2','c4','c5'):
    d=json.load(open('gpurun_out/r6y/%s.json'%w)); r=d['roofline']
    print(w, d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['alg_bytes_per_launch'], r['traffic_stale'], r['mfma_busy_frac'], d['hbm'].get('pmc_frac'), (d.get('cpu_baseline') or {}).get('value'))
PY
