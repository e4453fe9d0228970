# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6g: (1) fp32 BN elementwise passes (bn8: 8-wide fp32 apply / backward apply, two-in-flight
# bits apply) vs the product library on C2; (2) the bf16 8-wide applies with 4 in flight (ewu4) on
# C5; (3) the fp32 dgrad epilogue with 4 columns per thread (g1: 4-wave 3 + 5 rows; g2: + 8-wave
# tiles 4 late rows) on C2; interleaved on one box; then kernel tests on the new forms
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6g; mkdir -p $O
lib() { if [ $1 = base ]; then echo $PWD/tmrnet_amd/libtmr.so; else echo $PWD/tmrnet_amd/libtmr_$1.so; fi; }
for rep in 1 2; do
  for v in base bn8 g1 g2; do
    TMR_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 3
    python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']['per_kind']; print('c2', '$v', $rep, d['value'], d['ms_per_step'], r['conv_dgrad']['ms'], d['loss_last'])"
  done
  for v in base ewu4; do
    TMR_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline --no-roofline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 4
    python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5', '$v', $rep, d['value'], d['ms_per_step'], d['loss_last'])"
  done
done
for v in bn8 g1; do
  TMR_LIB_PATH=$(lib $v) timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -k "bn or parity or dgrad" > $O/pytest_$v.txt 2>&1
  echo "pytest rc=$?" >> $O/pytest_$v.txt
  tail -3 $O/pytest_$v.txt
done
