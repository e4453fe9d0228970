#!/bin/bash
# HBM traffic of one bench step: two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass on gfx950), kernel-trace only (no sys/runtime traces with --pmc), then
# scripts/pmc_summary.py -> gpurun_out/$PROF_NAME/pmc_traffic_<model>.json.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-pmc}
MODEL=${MODEL:-resnet50}
PRECISION=${PRECISION:-fp32}
TAG=$MODEL$([ "$PRECISION" = fp32 ] || echo _$PRECISION)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  # rocprofv3 (ROCm 7.2) can segfault in its own exit handlers after the results are written
  # (rc 139); the pass counts as done when the bench line and the counter CSV are there
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --model $MODEL --precision $PRECISION \
    > "$OUT/bench_$C.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && { [ $rc -ne 139 ] || ! grep -q '"metric"' "$OUT/bench_$C.log" || \
       [ -z "$(find "$OUT/$C" -name '*counter_collection*')" ]; }; then
    echo "pmc pass $C failed rc=$rc"; tail -5 "$OUT/bench_$C.log"; exit 1
  fi
done
python3 "$R/scripts/pmc_summary.py" "$OUT" --model $TAG > "$OUT/pmc_traffic_$TAG.json" && \
  cat "$OUT/pmc_traffic_$TAG.json"
