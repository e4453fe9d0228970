# BN partial reductions in one launch (last-arriving slab block finishes): full GPU suite, then a
# same-box C2 / C5 A/B against the previous build (libtmr_ab.so), interleaved, twice
set -o pipefail
O=gpurun_out/s5ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1 || exit 1
for rep in 1 2; do
  TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_ab.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --steps 15 > $O/c2_old_$rep.json 2> $O/c2_old_$rep.err || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --steps 15 > $O/c2_new_$rep.json 2> $O/c2_new_$rep.err || exit 1
  TMR_LIB_PATH=$PWD/tmrnet_amd/libtmr_ab.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_old_$rep.json 2> $O/c5_old_$rep.err || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_new_$rep.json 2> $O/c5_new_$rep.err || exit 1
done
