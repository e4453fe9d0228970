# round 5: dgrad epilogue A/B (whole-tile staging) + bf16 ensemble study
set -o pipefail
O=gpurun_out/s5d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "dgrad or bnbwd or g16 or resgrad or geometry_step or c2_geometry" tests/ > $O/pytest.txt 2>&1 || exit 1
B="timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --conv-table"
TMR_LIB_PATH=tmrnet_amd/libtmr_ab.so $B > $O/c2_head.json 2> $O/c2_head.err || exit 1
$B > $O/c2_new.json 2> $O/c2_new.err || exit 1
TMR_DGRAD32_WIDE_CFG=2 $B > $O/c2_new_w2.json 2> $O/c2_new_w2.err || exit 1
TMR_LIB_PATH=tmrnet_amd/libtmr_ab.so $B --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_head.json 2> $O/c5_head.err || exit 1
$B --precision bf16 --seq 30 --lfb 300 --steps 6 > $O/c5_new.json 2> $O/c5_new.err || exit 1
S="timeout -k 10 400 python -u scripts/bf16_grad_study.py --out $O"
$S --geo c5 --frames noise --variants fp32 --ensemble 4 --lrs 1e-5 --traj-variants fp32n,bf16_actoff,bf16_gradsoff > $O/study_c5_noise.txt 2>&1 || exit 1
$S --geo c4 --frames noise --variants fp32 --ensemble 4 --lrs 1e-5 --traj-variants fp32n,bf16_actoff > $O/study_c4_noise.txt 2>&1
