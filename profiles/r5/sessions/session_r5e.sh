set -o pipefail
O=gpurun_out/s5e; mkdir -p $O
S="timeout -k 10 400 python -u scripts/bf16_grad_study.py --out $O"
$S --geo c5 --frames noise --variants fp32 --ensemble 4 --lrs 3e-5 --traj-variants fp32,bf16 > $O/study_c5_noise.txt 2>&1 || exit 1
$S --geo c4 --frames noise --variants fp32 --ensemble 4 --lrs 3e-5 --traj-variants fp32,bf16 > $O/study_c4_noise.txt 2>&1
