# strided dgrads as one launch (chunks of 64 tiles per class): bit-identity tests, the A/B against
# per-class launches, then C2 / C5 bench lines
set -o pipefail
R=$PWD
O=$R/gpurun_out/s5al; mkdir -p $O
S=128:128:3:56,256:256:3:28,512:512:3:14,256:512:1:56,512:1024:1:28,1024:2048:1:14
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "parity_classes or fused_bn_backward or dgrad" > $O/pytest.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bf16_gpu.py tests/test_resnest_trunk_gpu.py -k "dgrad or trunk" > $O/pytest_bf16.txt 2>&1 || exit 1
for m in cl par; do
  F=""; [ $m = cl ] && F="--classes"
  timeout -k 10 200 python scripts/convbench.py --frames 1920 --reps 5 --io16 --bnbwd --kinds dgrad --only $S $F > $O/bf16_$m.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/convbench.py --frames 640 --reps 5 --wt32 --bnbwd --kinds dgrad --only $S $F > $O/f32_$m.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 > $O/c5.json 2> $O/c5.err
