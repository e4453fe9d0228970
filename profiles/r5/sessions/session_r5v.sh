# trunk.DS_DUAL on the ResNeSt trunk too: bit-identity (both trunks, fp32 / bf16), then a same-box
# C4 A/B (DS_DUAL flipped in-process before bench.py runs), interleaved, twice
set -o pipefail
O=gpurun_out/s5v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "ds_dual" > $O/pytest.txt 2>&1 || exit 1
B="--no-cpu-baseline --no-roofline --model resnest50 --precision bf16 --steps 10"
for rep in 1 2; do
  for d in False True; do
    timeout -k 10 200 python -u -c "import sys, runpy; import tmrnet_amd.trunk as t; t.DS_DUAL = $d; sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')" $B > $O/c4_${d}_$rep.json 2> $O/c4_${d}_$rep.err || exit 1
  done
done
