# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4x; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/test_direct3_gpu.py > $O/pytest_d3.txt 2>&1
rc=$?; echo "d3 rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest_d3.txt | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/scripts/probe/d3_probe.py 3 > $O/kt.log 2>&1 || exit 2
python3 - <<'PY'
import csv,glob,os
f=glob.glob(os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/r4x/kt/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    if 'd3' in r['Name']: print('%-70s %s %.3f ms'%(r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e6))
PY
cd $R
timeout -k 10 300 python bench.py --steps 10 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 5
python -c "import json;d=json.load(open('$O/c5.json'));r=d['roofline'];print('c5', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'), {k:v['ms'] for k,v in r.get('per_kind').items()})"
timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 4
python -c "import json;d=json.load(open('$O/c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'))"
