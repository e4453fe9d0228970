#!/bin/bash
# HBM traffic of one bench step: two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass on gfx950), kernel-trace only (no sys/runtime traces with --pmc), then
# scripts/pmc_summary.py -> gpurun_out/$PROF_NAME/pmc_traffic_<model>.json.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-pmc}
MODEL=${MODEL:-resnet50}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --model $MODEL \
    > "$OUT/bench_$C.log" 2>&1 || { echo "pmc pass $C failed rc=$?"; tail -5 "$OUT/bench_$C.log"; exit 1; }
done
python3 "$R/scripts/pmc_summary.py" "$OUT" --model $MODEL > "$OUT/pmc_traffic_$MODEL.json" && \
  cat "$OUT/pmc_traffic_$MODEL.json"
