set -e
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3g/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.txt 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r3g/bench_default.json 2> gpurun_out/r3g/bench_default.err
