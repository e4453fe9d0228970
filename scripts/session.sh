# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4q; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/test_direct3_gpu.py > $O/pytest_d3.txt 2>&1
rc=$?; echo "d3 rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_d3.txt | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 300 python bench.py --steps 6 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline --conv-table > $O/c4.json 2> $O/c4.err || exit 4
python -c "import json;d=json.load(open('$O/c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'), r.get('per_kind'))"
grep -E "112, 112, 32|224, 224" $O/c4.err
