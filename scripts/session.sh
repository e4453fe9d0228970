# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6c: compile-time epilogue forms of the 4-wave fused BN-backward dgrads (EpiForm) with
# more rows in flight once the accumulators are staged -- A/B against the product library, same
# box, interleaved; then the dgrad kernel tests on the leading variant
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6c; mkdir -p $O
for rep in 1 2; do
  for v in base fa fb fc; do
    if [ $v = base ]; then L=$PWD/tmrnet_amd/libtmr.so; else L=$PWD/tmrnet_amd/libtmr_$v.so; fi
    TMR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 2
    TMR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 3
    python -c "import json
for w in ('c5','c2'):
    d=json.load(open('$O/%s_${v}_$rep.json'%w)); r=d['roofline']['per_kind']
    print(w, '$v', $rep, d['value'], d['ms_per_step'], 'dgrad', r['conv_dgrad'], 'loss', d['loss_last'])"
  done
done
TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_fa.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_bf16_gpu.py -k "dgrad or bnbwd or g16" > $O/pytest_fa.txt 2>&1
echo "pytest rc=$?" >> $O/pytest_fa.txt
tail -4 $O/pytest_fa.txt
