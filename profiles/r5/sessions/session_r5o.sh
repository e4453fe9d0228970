# bf16 dY-operand prologue (trunk.FOLD16DY, A/B build): bit-identity against the explicit
# bn_bwd_apply8_a16 passes, then a same-box C5 A/B (interleaved, twice) with per-launch tables.
set -o pipefail
O=gpurun_out/s5o; mkdir -p $O
export TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_pro.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "fold16" > $O/pytest.txt 2>&1 || exit 1
B="--no-cpu-baseline --precision bf16 --seq 30 --lfb 300"
for f in 0 1; do
  TMR_FOLD16_DY=$f timeout -k 10 200 python -u bench.py $B --steps 3 --conv-table > $O/c5_dy${f}_tab.json 2> $O/c5_dy${f}_tab.err || exit 1
done
