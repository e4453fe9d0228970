# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: the forward statistics pass without per-row selects on whole tiles -- same-box A/B on
# the 1x1 forwards, the loss of short C5 / C2 runs against the previous build (bit-identity), the
# statistics tests
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6zc; mkdir -p $O
TMR_LIB_PATH=tmrnet_amd/libtmr_new.so timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/new.json > $O/new.log 2>&1 || exit 1
TMR_LIB_PATH=tmrnet_amd/libtmr.so timeout -k 10 300 python -u scripts/resdgrad_bench.py --frames 640 --kinds fwd --json $O/prev.json > $O/prev.log 2>&1 || exit 2
TMR_LIB_PATH=tmrnet_amd/libtmr_new.so timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_new.json 2> $O/c5_new.err || exit 3
TMR_LIB_PATH=tmrnet_amd/libtmr.so timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_prev.json 2> $O/c5_prev.err || exit 4
TMR_LIB_PATH=tmrnet_amd/libtmr_new.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c2_new.json 2> $O/c2_new.err || exit 5
TMR_LIB_PATH=tmrnet_amd/libtmr.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c2_prev.json 2> $O/c2_prev.err || exit 6
TMR_LIB_PATH=tmrnet_amd/libtmr_new.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_bf16_gpu.py -k "stats or y16 or storage or chunk" > $O/pytest.txt 2>&1 || exit 7
python - <<'PY'
import json
rows={}
for v in ('new','prev'):
    for r in json.load(open('gpurun_out/r6zc/%s.json'%v)):
        rows.setdefault((r['prec'],r['h'],r['N'],r['K']),{})[v]=r['ms']
for k,v in rows.items(): print(k, v)
for w in ('c5_new','c5_prev','c2_new','c2_prev'):
    d=json.load(open('gpurun_out/r6zc/%s.json'%w)); print(w, repr(d['loss_last']), d['value'])
PY
tail -2 $O/pytest.txt
