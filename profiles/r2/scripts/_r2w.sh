set -e
mkdir -p gpurun_out/r2w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2w/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2w/smoke.txt 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r2w/bench_default.json 2> gpurun_out/r2w/bench_default.err
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > gpurun_out/r2w/c2_bf16.json 2> gpurun_out/r2w/c2_bf16.err
