# one-pass BN backward of the downsample blocks' bn3 + downsample BN (trunk.DS_DUAL): bit-identity,
# then same-box C2 / C5 A/B (TMR_DS_DUAL=0/1, interleaved, twice)
set -o pipefail
O=gpurun_out/s5u; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "ds_dual" > $O/pytest.txt 2>&1 || exit 1
for rep in 1 2; do
  for d in 0 1; do
    TMR_DS_DUAL=$d timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --steps 15 > $O/c2_d${d}_$rep.json 2> $O/c2_d${d}_$rep.err || exit 1
    TMR_DS_DUAL=$d timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_d${d}_$rep.json 2> $O/c5_d${d}_$rep.err || exit 1
  done
done
