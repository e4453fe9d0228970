# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem or fused_bn_stats" -m gpu > $O/pytest_stem.txt 2>&1 || exit $?
TMR_STEM_DIRECT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --conv-table > $O/c2_stem.json 2> $O/c2_stem_table.txt || exit $?
TMR_STEM_DIRECT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --conv-table > $O/c2_nostem.json 2> $O/c2_nostem_table.txt || exit $?
TMR_STEM_DIRECT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2_stem2.json 2> $O/c2_stem2.err
echo "main rc=$?"
