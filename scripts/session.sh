# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# final-build PMC passes: C2 fp32, C4 bf16 (ResNeSt), C5 bf16 -> gpurun_out/r4f_pmc_*/pmc_traffic_*.json
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PROF_NAME=r4f_pmc_c2 MODEL=resnet50 PRECISION=fp32 SEQ=10 LFB=40 timeout -k 10 900 bash scripts/pmc.sh > gpurun_out/r4f_pmc_c2.log 2>&1 || { tail -5 gpurun_out/r4f_pmc_c2.log; exit 2; }
echo c2 done
PROF_NAME=r4f_pmc_c4 MODEL=resnest50 PRECISION=bf16 SEQ=10 LFB=40 timeout -k 10 900 bash scripts/pmc.sh > gpurun_out/r4f_pmc_c4.log 2>&1 || { tail -5 gpurun_out/r4f_pmc_c4.log; exit 3; }
echo c4 done
PROF_NAME=r4f_pmc_c5 MODEL=resnet50 PRECISION=bf16 SEQ=30 LFB=300 timeout -k 10 900 bash scripts/pmc.sh > gpurun_out/r4f_pmc_c5.log 2>&1 || { tail -5 gpurun_out/r4f_pmc_c5.log; exit 4; }
echo c5 done
ls gpurun_out/r4f_pmc_*/pmc_traffic_*.json
