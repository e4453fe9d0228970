# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: where the 1x1 forwards' time goes -- the product, without the statistics pass
# (TMR_FWD_EXP=1), without the y stores (2); timing only
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6zb; mkdir -p $O
timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/prod.json > $O/prod.log 2>&1 || exit 1
TMR_LIB_PATH=tmrnet_amd/libtmr_fx1.so timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/nostats.json > $O/nostats.log 2>&1 || exit 2
TMR_LIB_PATH=tmrnet_amd/libtmr_fx2.so timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/nostores.json > $O/nostores.log 2>&1 || exit 3
python - <<'PY'
import json
rows={}
for v in ('prod','nostats','nostores'):
    for r in json.load(open('gpurun_out/r6zb/%s.json'%v)):
        rows.setdefault((r['prec'],r['h'],r['N'],r['K']),{})[v]=r['ms']
for k,v in rows.items(): print(k, v)
PY
