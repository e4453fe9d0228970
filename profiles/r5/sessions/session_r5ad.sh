# round 5 final build (3): full GPU suite, the A/B-build fold tests, smoke, C2 / C4 / C5 benches
set -o pipefail
O=gpurun_out/s5ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1
echo "pytest rc=$?" >> $O/pytest.txt
TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_pro.so timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "fold" > $O/pytest_fold_ab.txt 2>&1
echo "pytest rc=$?" >> $O/pytest_fold_ab.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python -u bench.py --model resnest50 --precision bf16 --steps 10 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
