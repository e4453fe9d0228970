# A/B of the round-5 tile rules (TMR_TILE_RULE=1: bf16 wgrads 128x128 8-wave / 256x256 16-wave
# by shape, fp32 forwards keep 256x256 at >= 224 tiles) on the C2 / C4 / C5 train steps,
# interleaved, then the conv parity tests on the new rules.
set -o pipefail
O=gpurun_out/s5m; mkdir -p $O
B="--no-cpu-baseline --no-roofline"
for rep in 1 2; do
  for r in 1 0; do
    TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --steps 15 > $O/c2_r${r}_$rep.json 2> $O/c2_r${r}_$rep.err || exit 1
    TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --model resnest50 --precision bf16 --steps 10 > $O/c4_r${r}_$rep.json 2> $O/c4_r${r}_$rep.err || exit 1
    TMR_TILE_RULE=$r timeout -k 10 200 python -u bench.py $B --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_r${r}_$rep.json 2> $O/c5_r${r}_$rep.err || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_bf16_gpu.py tests/test_geometry_gpu.py > $O/pytest.txt 2>&1 || exit 1
