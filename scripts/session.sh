# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# final build, part 1: GPU test suite + smoke, then PMC traffic records of C2 (fp32), C4 and C5 (bf16)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4h_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4h_smoke.log 2>&1 || { tail -3 gpurun_out/r4h_smoke.log; exit 9; }
tail -1 gpurun_out/r4h_smoke.log
PROF_NAME=r4h_pmc_c2 MODEL=resnet50 PRECISION=fp32 SEQ=10 LFB=40 bash scripts/pmc.sh > gpurun_out/r4h_pmc_c2.txt 2>&1 || { tail -5 gpurun_out/r4h_pmc_c2.txt; exit 2; }
echo c2 done
PROF_NAME=r4h_pmc_c4 MODEL=resnest50 PRECISION=bf16 SEQ=10 LFB=40 bash scripts/pmc.sh > gpurun_out/r4h_pmc_c4.txt 2>&1 || { tail -5 gpurun_out/r4h_pmc_c4.txt; exit 3; }
echo c4 done
PROF_NAME=r4h_pmc_c5 MODEL=resnet50 PRECISION=bf16 SEQ=30 LFB=300 bash scripts/pmc.sh > gpurun_out/r4h_pmc_c5.txt 2>&1 || { tail -5 gpurun_out/r4h_pmc_c5.txt; exit 4; }
echo c5 done
