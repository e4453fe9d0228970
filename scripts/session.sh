# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# wgrad split-K target sweep (TMR_WGRAD_TARGET) after the workspace-query fix
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4h_wgt; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_bf16_gpu.py -k "wgrad or conv" > $O/t.log 2>&1; rc=$?; tail -1 $O/t.log; [ $rc -eq 0 ] || exit $rc
for t in 512 768 1024 512 768 1024; do
  TMR_WGRAD_TARGET=$t timeout -k 10 300 python bench.py --steps 10 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline > $O/c5_$t.json 2> $O/c5_$t.err || exit 4
  python -c "import json;d=json.load(open('$O/c5_$t.json'));print('c5 target $t', d['value'], d['ms_per_step'], d['roofline']['per_kind']['conv_wgrad_bf16']['ms'])"
done
for t in 512 768 1024; do
  TMR_WGRAD_TARGET=$t timeout -k 10 300 python bench.py --steps 10 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline > $O/c4_$t.json 2> $O/c4_$t.err || exit 3
  python -c "import json;d=json.load(open('$O/c4_$t.json'));print('c4 target $t', d['value'], d['ms_per_step'])"
  TMR_WGRAD_TARGET=$t timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > $O/c2_$t.json 2> $O/c2_$t.err || exit 2
  python -c "import json;d=json.load(open('$O/c2_$t.json'));print('c2 target $t', d['value'], d['ms_per_step'])"
done
