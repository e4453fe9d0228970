# weight layouts of a step in one launch (ops.layout_session): equality tests, model parity tests,
# then same-box C2 / C5 / C4 A/B (sessions turned off in-process for the reference), interleaved
set -o pipefail
O=gpurun_out/s5ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_compat_gpu.py tests/test_resnest_gpu.py -k "layout or parity or compat or resnest" > $O/pytest.txt 2>&1 || exit 1
run() {  # name, sessions (True/False), bench args...
  local n=$1 on=$2; shift 2
  timeout -k 10 200 python -u -c "import sys, runpy; import tmrnet_amd.ops as o; o.LAYOUT_SESSIONS = $on; sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')" "$@" > $O/$n.json 2> $O/$n.err
}
for rep in 1 2; do
  for on in False True; do
    run c2_${on}_$rep $on --no-cpu-baseline --no-roofline --steps 15 || exit 1
    run c5_${on}_$rep $on --no-cpu-baseline --no-roofline --precision bf16 --seq 30 --lfb 300 --steps 6 || exit 1
    run c4_${on}_$rep $on --no-cpu-baseline --no-roofline --model resnest50 --precision bf16 --steps 10 || exit 1
  done
done
