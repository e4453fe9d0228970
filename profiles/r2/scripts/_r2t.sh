set -e
mkdir -p gpurun_out/r2t
PROF_NAME=r2t/pmc bash scripts/pmc.sh > gpurun_out/r2t/pmc.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2t/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2t/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2t/prof_bench.err || [ $? -eq 139 ]
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/r2t/bench_default.json 2> gpurun_out/r2t/bench_default.err
