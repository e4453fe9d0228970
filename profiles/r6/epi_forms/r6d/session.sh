# one GPU session (edited per call; the records it writes are copied into profiles/<round>/)
# round 6d: epilogue forms, second sweep -- fa (round-6c leader), fd (bf16: 5 rows before the main
# loop + 3 after staging), fa with the fp32 N >= 512 dgrads on the 4-wave tile
# (TMR_DGRAD32_WIDE_CFG=2), fe (8-wave tiles: 2 rows in flight after staging, spills)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6d; mkdir -p $O
for rep in 1 2; do
  for v in fa fd fa2 fe; do
    L=$PWD/tmrnet_amd/libtmr_${v%2}.so; W=7
    [ $v = fa2 ] && W=2
    TMR_DGRAD32_WIDE_CFG=$W TMR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --precision bf16 --seq 30 --lfb 300 --steps 6 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 2
    TMR_DGRAD32_WIDE_CFG=$W TMR_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --conv-table > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 3
  done
done
python - <<'PY'
import json
for w in ('c5','c2'):
    for v in ('fa','fd','fa2','fe'):
        for rep in (1,2):
            d=json.load(open('gpurun_out/r6d/%s_%s_%d.json'%(w,v,rep)))
            dg=[x for k,x in d['roofline']['per_kind'].items() if 'dgrad' in k][0]
            print(w,v,rep,d['value'],d['ms_per_step'],'dgrad',dg['ms'],dg['tflops'],'loss',d['loss_last'])
PY
