set -o pipefail
O=gpurun_out/s5j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_parity_gpu.py -k "side_stream" > $O/pytest.txt 2>&1 || exit 1
B="timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline"
$B > $O/c2_s0.json 2> $O/c2_s0.err || exit 1
TMR_WGRAD_STREAM=1 $B > $O/c2_s1.json 2> $O/c2_s1.err || exit 1
$B > $O/c2_s0b.json 2> $O/c2_s0b.err || exit 1
TMR_WGRAD_STREAM=1 $B > $O/c2_s1b.json 2> $O/c2_s1b.err || exit 1
B5="timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --warmup 3 --no-cpu-baseline"
$B5 > $O/c5_s0.json 2> $O/c5_s0.err || exit 1
TMR_WGRAD_STREAM=1 $B5 > $O/c5_s1.json 2> $O/c5_s1.err || exit 1
