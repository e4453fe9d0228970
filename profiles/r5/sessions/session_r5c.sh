set -o pipefail
mkdir -p gpurun_out/s5c
S="timeout -k 10 400 python -u scripts/bf16_grad_study.py --out gpurun_out/s5c"
$S --geo c5 --frames noise --variants fp32 --ensemble 4 --lrs 1e-5 --traj-variants fp32n,bf16_actoff,bf16_gradsoff > gpurun_out/s5c/study_c5_noise.txt 2>&1 || exit 1
$S --geo c4 --frames noise --variants fp32 --ensemble 4 --lrs 1e-5 --traj-variants fp32n,bf16_actoff > gpurun_out/s5c/study_c4_noise.txt 2>&1
