# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests/test_resnest_trunk_gpu.py tests/test_resnest_gpu.py tests/test_geometry_gpu.py -k "c4 or resnest or split or grouped or attention or avgpool" > $O/pytest.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.txt | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for g in 256 1024; do
TMR_SPLAT_GAP_BT=$g timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4_g$g.json 2> $O/c4_g$g.err || exit 4
python -c "import json;d=json.load(open('$O/c4_g$g.json'));r=d['roofline'];print('c4 gapbt=$g', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'))"
done
PROF_NAME=r4t_c4 STEPS=3 BENCH_ARGS="--precision bf16 --model resnest50 --seq 10 --lfb 40" bash scripts/profile.sh > $O/prof.txt 2>&1 || exit 3
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r4t_c4/**/*kernel_stats*.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total ms/pass', tot/1e6/5)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:24]:
    print('%-70s %5s %8.2f'%(r['Name'][:70],r['Calls'],float(r['TotalDurationNs'])/1e6/5))
PY
