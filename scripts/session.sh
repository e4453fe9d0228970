# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_geometry_gpu.py tests/test_resnest_trunk_gpu.py tests/test_resnest_gpu.py tests/test_bf16_vs_fp32_gpu.py tests/test_bf16_gpu.py -k "c4 or resnest" > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" $O/pytest.txt | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for f in 0 1; do
  TMR_BF16_RESGRAD=$f timeout -k 10 300 python bench.py --steps 10 --model resnest50 --precision bf16 --no-cpu-baseline > $O/c4_r16_$f.json 2> $O/c4_r16_$f.err || exit 3
  python -c "import json;d=json.load(open('$O/c4_r16_$f.json'));r=d['roofline'];print('r16=$f', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['per_kind'])"
done
# stats-epilogue cost of the store-bound 1x1 expansions (bf16 operands, C5 frames)
for m in "" "--stats" "--y16"; do
  timeout -k 10 200 python scripts/convbench.py --frames 1920 --io16 --kinds fwd --only 64:256:1:56,128:512:1:28,256:1024:1:14,64:64:1:56 $m > $O/cb_fwd$m.txt 2>&1 || exit 5
  echo "== $m"; grep -v TOTAL $O/cb_fwd$m.txt | tail -5
done
