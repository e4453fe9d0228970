#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC here: counters go in their own pass)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-prof}
mkdir -p "$OUT"
# build stamp: the sha256 of the library these kernel stats come from (bench.py build_sha)
python3 -c "import sys; sys.path.insert(0, '$R/scripts'); import pmc_summary as p; print(p.lib_sha('$R/tmrnet_amd/libtmr.so'))" > "$OUT/build_sha.txt"
cd /tmp && export TMPDIR=/tmp
export TMR_EXIT_MAPS="$OUT/exit_maps.txt"
# (the benchmarked step's persistent LSTM included: see scripts/pmc.sh)
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$R/bench.py" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 "$OUT/bench.log"
find "$OUT" -name "*stats*" | head
exit $rc
