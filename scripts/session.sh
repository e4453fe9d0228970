# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 600 python bench.py > $O/c2_default.json 2> $O/c2_default.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --model resnest50 --precision bf16 > $O/c4.json 2> $O/c4.err
echo "main rc=$?"
