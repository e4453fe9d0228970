#!/bin/bash
# HBM traffic of one bench step: two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass on gfx950), kernel-trace only (no sys/runtime traces with --pmc), then
# scripts/pmc_summary.py -> gpurun_out/$PROF_NAME/pmc_traffic_<model>.json.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-pmc}
MODEL=${MODEL:-resnet50}
PRECISION=${PRECISION:-fp32}
# the record's name keys the workload (bench.py load_traffic): model, precision, seq, LFB
TAG=${TAG:-${MODEL}_${PRECISION}_s${SEQ:-10}_l${LFB:-40}}
BENCH_ARGS="${BENCH_ARGS} --seq ${SEQ:-10} --lfb ${LFB:-40}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# Profiled runs take the benchmarked step's persistent LSTM (round 5: a plain launch after an
# occupancy check; the cooperative launch of rounds 2-4 made the process fault at exit under
# rocprofv3, profiles/r3/exit_probe/, so those profiles used the per-step path).
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --model $MODEL --precision $PRECISION ${BENCH_ARGS} \
    > "$OUT/bench_$C.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pmc pass $C failed rc=$rc"; tail -5 "$OUT/bench_$C.log"; exit 1
  fi
done
# MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over every SIMD) against the kernel's
# cycles (GRBM_GUI_ACTIVE summed over the 8 XCDs, / 8) x 1024 SIMDs -- one SQ and one GRBM counter
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d "$OUT/MFMA" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --model $MODEL --precision $PRECISION ${BENCH_ARGS} \
  > "$OUT/bench_MFMA.log" 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "pmc pass MFMA failed rc=$rc"; tail -5 "$OUT/bench_MFMA.log"; exit 1; fi
python3 "$R/scripts/pmc_summary.py" "$OUT" --model $TAG > "$OUT/pmc_traffic_$TAG.json" && \
  cat "$OUT/pmc_traffic_$TAG.json"
