# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6b: bf16 ensemble vs emulation, the full-size bf16 gradient acceptance (projection floor,
# lr 1e-5 trajectory), then the stall-counter passes of the conv kernels at C5
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread \
  tests/test_bf16_ensemble_gpu.py tests/test_bf16_grads_gpu.py > $O/pytest.txt 2>&1
echo "pytest rc=$?" >> $O/pytest.txt
tail -15 $O/pytest.txt
cp gpurun_out/bf16_ensemble_*.json gpurun_out/bf16_grads_*.json $O/ 2>/dev/null
PROF_NAME=r6b/pmc_stall_c5 bash scripts/pmc_stall.sh > $O/pmc_stall_c5.txt 2>&1 || { tail -20 $O/pmc_stall_c5.txt; exit 3; }
tail -5 $O/pmc_stall_c5.txt
