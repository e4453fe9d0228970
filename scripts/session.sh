# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --model resnest50 --precision bf16 > $O/c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2.json 2> $O/c2.err && \
TMR_DS_FIRST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2_dsfirst.json 2> $O/c2_dsfirst.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/c2_again.json 2> $O/c2_again.err
echo "main rc=$?"
cd /tmp && export TMPDIR=/tmp
for m in plain pinned lib conv lstm step; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/probe_$m -o run -- python3 $R/scripts/exit_probe.py $m > $R/$O/probe_$m.log 2>&1
  rc=$?; echo "probe $m rc=$rc"
  if [ $rc -ne 0 ]; then break; fi
done
