#!/bin/bash
# Stall / issue counters of the conv engine's kernels over one bench step (the
# bf16 dgrad gemm16_kernel<1,128,128,2,2> that dominates C4 / C5).  One rocprofv3 PMC pass per
# counter set (each within gfx950's per-block slots: 8 SQ, 2 GRBM, 4 TCP, 2 TA, 2 TD), kernel
# trace only, the conv kernels only (--kernel-include-regex), every pass under its own time
# limit; then scripts/pmc_stall_summary.py -> gpurun_out/$PROF_NAME/pmc_stall.json.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-pmc_stall}
BENCH_ARGS=${BENCH_ARGS:---precision bf16 --seq 30 --lfb 300}
REGEX=${REGEX:-gemm16}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
declare -a PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_VMEM SQ_INSTS_MFMA TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TD_TD_BUSY_sum"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  # keep only the counters this box lists (an unknown name fails the pass)
  keep=""
  for c in $P; do
    base=${c%_sum}
    if grep -q "\b$c\b\|\b$base\b" "$OUT/avail.txt"; then keep="$keep $c"; fi
  done
  echo "pass $i:$keep"
  [ -z "$keep" ] && continue
  timeout -s KILL 300 rocprofv3 --pmc $keep --kernel-trace --kernel-include-regex "$REGEX" \
    --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline ${BENCH_ARGS} \
    > "$OUT/bench_p$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 "$OUT/bench_p$i.log"; exit 1; fi
done
python3 "$R/scripts/pmc_stall_summary.py" "$OUT" > "$OUT/pmc_stall.json" && head -c 3000 "$OUT/pmc_stall.json"
