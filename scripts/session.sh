# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/test_direct3_gpu.py > $O/pytest_d3.txt 2>&1
rc=$?; echo "d3 rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest_d3.txt | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests/test_resnest_trunk_gpu.py tests/test_resnest_gpu.py tests/test_geometry_gpu.py tests/test_bf16_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.txt | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline --conv-table > $O/c5.json 2> $O/c5.err || exit 5
python -c "import json;d=json.load(open('$O/c5.json'));r=d['roofline'];print('c5', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'), {k:v['ms'] for k,v in r.get('per_kind').items()})"
grep -E "56, 56, 64, 64, 3" $O/c5.err | head -9
for g in 256 1024; do
TMR_SPLAT_GAP_BT=$g timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4_g$g.json 2> $O/c4_g$g.err || exit 4
python -c "import json;d=json.load(open('$O/c4_g$g.json'));r=d['roofline'];print('c4 gapbt=$g', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'))"
done
