set -o pipefail
O=gpurun_out/s5h; mkdir -p $O
export TMR_LIB_PATH=tmrnet_amd/libtmr_pro.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fold" > $O/pytest_fold.txt 2>&1 || exit 1
B="timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --warmup 3 --no-cpu-baseline --conv-table"
$B > $O/c5_pro.json 2> $O/c5_pro.err || exit 1
TMR_FOLD16=1 $B > $O/c5_fold16.json 2> $O/c5_fold16.err || exit 1
$B > $O/c5_pro2.json 2> $O/c5_pro2.err || exit 1
TMR_FOLD16=1 $B > $O/c5_fold16b.json 2> $O/c5_fold16b.err || exit 1
