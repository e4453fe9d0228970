# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_modules_gpu.py tests/test_compat_gpu.py tests/test_ddp_gpu.py tests/test_bf16_vs_fp32_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest.txt
mv gpurun_out/bf16_vs_fp32_*.json $O/
exit $rc
