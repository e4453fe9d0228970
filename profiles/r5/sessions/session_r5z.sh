# final build: the dual BN-backward op tests, then the run-to-run spread of the three benches on
# one box (C2 default command x3, C4 / C5 x2), traffic read from the committed PMC records
set -o pipefail
O=gpurun_out/s5z; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "parts_ds_op or ds_dual" > $O/pytest.txt 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/c2_$rep.json 2> $O/c2_$rep.err || exit 1
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnest50 --precision bf16 --steps 10 --no-cpu-baseline > $O/c4_$rep.json 2> $O/c4_$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5_$rep.json 2> $O/c5_$rep.err || exit 1
done
