set -e
mkdir -p gpurun_out/r2p
PROF_NAME=r2p/pmc bash scripts/pmc.sh > gpurun_out/r2p/pmc.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2p/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2p/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2p/prof_bench.err || [ $? -eq 139 ]
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/r2p/bench_default.json 2> gpurun_out/r2p/bench_default.err
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2p/smoke.txt 2>&1
