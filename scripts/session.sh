set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_resnest_trunk_gpu.py tests/test_resnest_gpu.py tests/test_bf16_gpu.py tests/test_geometry_gpu.py tests/test_kernels_gpu.py -k "split or resnest or geometry or c4 or fused_bn_backward or grouped" > gpurun_out/r4c/pytest.txt 2>&1
echo "pytest rc=$?"
timeout -k 10 200 python scripts/convbench.py --kinds dgrad --bnbwd --wt32 --dgrad-beta 1 --reps 4 > gpurun_out/r4c/cb_new.txt 2>&1 && \
TMR_LIB_PATH=tmrnet_amd/libtmr_ab.so timeout -k 10 200 python scripts/convbench.py --kinds dgrad --bnbwd --wt32 --dgrad-beta 1 --reps 4 > gpurun_out/r4c/cb_old.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r4c/c2.json 2> gpurun_out/r4c/c2.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > gpurun_out/r4c/c4.json 2> gpurun_out/r4c/c4.err
echo "rc=$?"
