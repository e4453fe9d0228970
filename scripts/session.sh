# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" -m gpu > $O/pytest_stem.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --conv-table > $O/c2_table.json 2> $O/c2_table.txt && \
timeout -k 10 600 python bench.py > $O/c2_default.json 2> $O/c2_default.err
echo "main rc=$?"
