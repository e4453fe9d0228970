# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/grad_ratios.jsonl
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests/test_geometry_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "rc=$rc"; grep -E "passed|failed|FAILED" $O/pytest.txt | tail -5
cat gpurun_out/grad_ratios.jsonl; for f in gpurun_out/geometry_*logits.json; do echo $f; tr -d '\n ' < $f; echo; done
exit $rc
