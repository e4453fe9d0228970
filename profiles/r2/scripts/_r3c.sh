set -e
mkdir -p gpurun_out/r3c
for t in 256 512 1024 2048; do
  TMR_WGRAD_TARGET=$t timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r3c/bench_t$t.json 2> gpurun_out/r3c/bench_t$t.err
done
