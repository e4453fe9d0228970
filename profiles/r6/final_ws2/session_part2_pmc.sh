# round 6 final build (wave-specialised dgrad), part 2: PMC traffic records (FETCH_SIZE, WRITE_SIZE, MFMA busy) of C2 / C4 /
# C5 stamped with the library's sha (bench.py reads them: traffic, mfma_busy_frac, hbm.pmc_*)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PROF_NAME=r6x/pmc_c2 MODEL=resnet50 PRECISION=fp32 SEQ=10 LFB=40 bash scripts/pmc.sh > gpurun_out/pmc_c2.txt 2>&1 || { tail -5 gpurun_out/pmc_c2.txt; exit 1; }
PROF_NAME=r6x/pmc_c4 MODEL=resnest50 PRECISION=bf16 SEQ=10 LFB=40 bash scripts/pmc.sh > gpurun_out/pmc_c4.txt 2>&1 || { tail -5 gpurun_out/pmc_c4.txt; exit 2; }
PROF_NAME=r6x/pmc_c5 MODEL=resnet50 PRECISION=bf16 SEQ=30 LFB=300 bash scripts/pmc.sh > gpurun_out/pmc_c5.txt 2>&1 || { tail -5 gpurun_out/pmc_c5.txt; exit 3; }
for w in c2 c4 c5; do python3 -c "
import json,glob
f=glob.glob('gpurun_out/r6x/pmc_$w/pmc_traffic_*.json')[0]; d=json.load(open(f))
fam=d['families']; tot=sum(v['hbm_bytes_per_step'] for v in fam.values())
print('$w', f, d['build_sha'], round(tot/1e9,1), 'GB/step')"; done
