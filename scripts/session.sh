# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6a: the new / changed GPU tests (LSTM recovery, layout lifetime, DDP diagnostics, bf16
# ensemble vs emulation, 8-wide pool kernels), then a short C2 bench
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_modules_gpu.py tests/test_ddp_gpu.py tests/test_stem_pool8_gpu.py \
  "tests/test_kernels_gpu.py::test_layout_sessions_model_lifetime" \
  "tests/test_kernels_gpu.py::test_weight_layout_sessions" \
  tests/test_bf16_ensemble_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 2; }
tail -5 $O/pytest.txt
cp gpurun_out/bf16_ensemble_*.json gpurun_out/lstm_resident_kernel.json $O/ 2>/dev/null
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
python -c "import json;d=json.load(open('$O/bench_c2.json'));print(d['value'], d['ms_per_step'], d['ranks'])"
