# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/test_direct3_gpu.py tests/test_resnest_trunk_gpu.py > $O/pytest_d3.txt 2>&1
rc=$?; echo "d3 rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest_d3.txt | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests/test_geometry_gpu.py -k c4 tests/test_bf16_vs_fp32_gpu.py -k c4 > $O/pytest_c4.txt 2>&1
rc=$?; echo "c4 tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest_c4.txt | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 6 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline --conv-table > $O/c4.json 2> $O/c4.err || exit 4
python -c "import json;d=json.load(open('$O/c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'), r.get('per_kind'))"
grep -E "112, 112, 32|224, 224" $O/c4.err
