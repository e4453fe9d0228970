# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.txt | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TMR_LIB_PATH=tmrnet_amd/libtmr_pro.so timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k fold > $O/pytest_fold.txt 2>&1
rc=$?; echo "fold rc=$rc"; grep -E "FAIL|ERROR|passed|failed|skipped" $O/pytest_fold.txt | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.txt
