# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: stall counters of the wave-specialised dgrad beside the engine's dgrad (C5 and C2 steps)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PROF_NAME=r6s/pmc_stall_c5 REGEX="dgrad_ws|gemm16_kernel" bash scripts/pmc_stall.sh > gpurun_out/pmc_stall_c5.txt 2>&1 || { tail -5 gpurun_out/pmc_stall_c5.txt; exit 1; }
PROF_NAME=r6s/pmc_stall_c2 REGEX="dgrad_ws|gemm16_kernel" BENCH_ARGS="--precision fp32 --seq 10 --lfb 40" bash scripts/pmc_stall.sh > gpurun_out/pmc_stall_c2.txt 2>&1 || { tail -5 gpurun_out/pmc_stall_c2.txt; exit 2; }
python3 - <<'PY'
import json
for c in ('c5','c2'):
    d=json.load(open('gpurun_out/r6s/pmc_stall_%s/pmc_stall.json'%c))
    for k,v in d.items():
        if 'dgrad_ws' in k or 'gemm16_kernel<1' in k:
            print(c, k[:60], {x: v.get(x) for x in ('frac_SQ_WAIT_ANY','frac_SQ_WAIT_INST_ANY','frac_SQ_ACTIVE_INST_ANY','mfma_busy_frac','lds_conflict_frac','TD_TD_BUSY_sum','launch_records')})
PY
