# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: the final build's GPU suite and smoke once more, on another box (stability check)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6zd; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1
echo "pytest rc=$?" >> $O/pytest.txt
tail -3 $O/pytest.txt
grep -E "FAILED|ERROR" $O/pytest.txt | head -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
