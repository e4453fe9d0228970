# strided dgrads: every stride-parity class in one launch vs one launch per class (A/B, one box);
# bit-identity tests first
set -o pipefail
R=$PWD
O=$R/gpurun_out/s5ai; mkdir -p $O
S=128:128:3:56,256:256:3:28,512:512:3:14,256:512:1:56,512:1024:1:28,1024:2048:1:14
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "parity_classes or fused_bn_backward or dgrad" > $O/pytest.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bf16_gpu.py -k "dgrad" > $O/pytest_bf16.txt 2>&1 &&
for cl in 0 1; do
  F=""; [ $cl = 1 ] && F="--classes"
  timeout -k 10 200 python scripts/convbench.py --frames 1920 --reps 5 --io16 --bnbwd --kinds dgrad --only $S $F > $O/bf16_cl$cl.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/convbench.py --frames 640 --reps 5 --wt32 --bnbwd --kinds dgrad --only $S $F > $O/f32_cl$cl.log 2>&1 || exit 1
done
