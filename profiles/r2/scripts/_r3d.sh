set -e
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3d/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d/smoke.txt 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r3d/bench_default.json 2> gpurun_out/r3d/bench_default.err
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --seq 30 --lfb 300 > gpurun_out/r3d/c5_bf16.json 2> gpurun_out/r3d/c5_bf16.err
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --model resnest50 > gpurun_out/r3d/c4_bf16.json 2> gpurun_out/r3d/c4_bf16.err
timeout -k 10 300 python bench.py --no-cpu-baseline --model resnest50 > gpurun_out/r3d/c4_fp32.json 2> gpurun_out/r3d/c4_fp32.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3d/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3d/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3d/prof_bench.err || [ $? -eq 139 ]
