set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2l/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2l/smoke.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r2l/bench_default.json 2> gpurun_out/r2l/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2l/prof_bf16 -o run -- python bench.py --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2l/prof_bf16.log 2>&1
