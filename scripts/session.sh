# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# final build, part 2: the bench lines (traffic from profiles/r4/) and rocprofv3 kernel stats
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err || exit 2
timeout -k 10 300 python bench.py --steps 20 --precision bf16 --model resnest50 --seq 10 --lfb 40 --no-cpu-baseline --conv-table > $O/bench_c4.json 2> $O/bench_c4.err || exit 3
timeout -k 10 400 python bench.py --steps 20 --precision bf16 --seq 30 --lfb 300 --no-cpu-baseline --conv-table > $O/bench_c5.json 2> $O/bench_c5.err || exit 4
for c in c2_default c4 c5; do python -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r.get('build_sha'), r.get('traffic_stale'), r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))"; done
PROF_NAME=r4i_prof_c2 STEPS=3 BENCH_ARGS="" bash scripts/profile.sh > $O/prof_c2.txt 2>&1 || exit 5
PROF_NAME=r4i_prof_c4 STEPS=3 BENCH_ARGS="--precision bf16 --model resnest50 --seq 10 --lfb 40" bash scripts/profile.sh > $O/prof_c4.txt 2>&1 || exit 6
PROF_NAME=r4i_prof_c5 STEPS=3 BENCH_ARGS="--precision bf16 --seq 30 --lfb 300" bash scripts/profile.sh > $O/prof_c5.txt 2>&1 || exit 7
echo profiles done
