# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4k; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_bf16_gpu.py tests/test_geometry_gpu.py tests/test_bf16_vs_fp32_gpu.py -k "stem or bf16 or c5" > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.txt | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 6 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline --conv-table > $O/c5.json 2> $O/c5.err || exit 3
python -c "import json;d=json.load(open('$O/c5.json'));r=d['roofline'];print('c5', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['per_kind'])"
grep "224, 224" $O/c5.err
