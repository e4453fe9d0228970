# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "bits" tests/test_resnest_trunk_gpu.py tests/test_resnest_gpu.py tests/test_geometry_gpu.py -k "bits or c4 or resnest or split or grouped or attention" > $O/pytest.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/pytest.txt | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do for b in 0 1; do
TMR_RELU_BITS16=$b timeout -k 10 300 python bench.py --steps 10 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline --conv-table > $O/c5_b${b}_$rep.json 2> $O/c5_b${b}_$rep.err || exit 5
python -c "import json;d=json.load(open('$O/c5_b${b}_$rep.json'));r=d['roofline'];print('c5 bits16=$b', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'), {k:v['ms'] for k,v in r.get('per_kind').items()})"
done; done
for s8 in 0 1; do
TMR_SPLAT8=$s8 timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4_s$s8.json 2> $O/c4_s$s8.err || exit 4
python -c "import json;d=json.load(open('$O/c4_s$s8.json'));r=d['roofline'];print('c4 splat8=$s8', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'))"
done
TMR_RELU_BITS16=1 timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4_b1.json 2> $O/c4_b1.err || exit 4
python -c "import json;d=json.load(open('$O/c4_b1.json'));r=d['roofline'];print('c4 bits16=1 splat8=1', d['value'], d['ms_per_step'], r.get('conv_ms_per_step'))"
