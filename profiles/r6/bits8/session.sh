# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6: the fp32 forward BN + ReLU + mask bits 8 elements per thread -- its tests, then C2 A/B
# against the 4-wide form (libtmr_bits4.so), interleaved
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "relu_bits or fused_bn_backward" tests/test_dgrad_ws_gpu.py > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_b8_a.json 2> $O/c2_b8_a.err || exit 2
TMR_LIB_PATH=tmrnet_amd/libtmr_bits4.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_b4_a.json 2> $O/c2_b4_a.err || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_b8_b.json 2> $O/c2_b8_b.err || exit 4
TMR_LIB_PATH=tmrnet_amd/libtmr_bits4.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_b4_b.json 2> $O/c2_b4_b.err || exit 5
python - <<'PY'
import json
for w in ('c2_b8_a','c2_b4_a','c2_b8_b','c2_b4_b'):
    d=json.load(open('gpurun_out/r6v/%s.json'%w))
    print(w, d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
