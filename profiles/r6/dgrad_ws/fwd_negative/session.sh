# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: the forward view of the wave-specialised kernel -- tests, then the 1x1 forwards with
# it and with the engine's tiles
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dgrad_ws_gpu.py > $O/pytest_ws.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/fwd_ws.json > $O/fwd_ws.log 2>&1 || exit 2
timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --tiles --json $O/fwd_tiles.json > $O/fwd_tiles.log 2>&1 || exit 3
python - <<'PY'
import json
rows={}
for v in ('fwd_ws','fwd_tiles'):
    for r in json.load(open('gpurun_out/r6z/%s.json'%v)):
        rows.setdefault((r['prec'],r['kind'],r['h'],r['N'],r['K']),{})[v]=(r['ms'], r['GBps'])
for k,v in rows.items(): print(k, v)
PY
