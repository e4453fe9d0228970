# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6 final build (wave-specialised dgrad on raw barriers, 8-wide fp32 bits apply, paired ds8), part 1: full GPU suite, smoke, C2 / C4 / C5 benches, rocprofv3 kernel stats
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1
echo "pytest rc=$?" >> $O/pytest.txt
tail -3 $O/pytest.txt
grep -E "FAILED|ERROR" $O/pytest.txt | head -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/c2.json 2> $O/c2.err || exit 2
timeout -k 10 300 python -u bench.py --model resnest50 --precision bf16 --steps 10 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 3
timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 4
python - <<'PY'
import json
for w in ('c2','c4','c5'):
    d=json.load(open('gpurun_out/r6w/%s.json'%w)); r=d['roofline']
    print(w, d['value'], d['ms_per_step'], r['frac'], r['build_sha'], {k: v['ms'] for k, v in r['per_kind'].items()}, (d.get('cpu_baseline') or {}).get('value'))
PY
PROF_NAME=r6w/prof_c2 STEPS=3 BENCH_ARGS="" bash scripts/profile.sh > $O/prof_c2.txt 2>&1 || exit 5
PROF_NAME=r6w/prof_c4 STEPS=3 BENCH_ARGS="--precision bf16 --model resnest50 --seq 10 --lfb 40" bash scripts/profile.sh > $O/prof_c4.txt 2>&1 || exit 6
PROF_NAME=r6w/prof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh > $O/prof_c5.txt 2>&1 || exit 7
echo profiles done
