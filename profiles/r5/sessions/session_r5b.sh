set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5b/pytest.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r5b/pytest.txt
S="timeout -k 10 300 python -u scripts/bf16_grad_study.py --out gpurun_out/r5b"
$S --geo c5 --frames noise --variants fp32,fp32p,fp32xb,bf16,bf16_actoff --lrs 1e-5,1e-4 --traj-variants fp32,fp32xb,bf16 > gpurun_out/r5b/study_c5_noise.txt 2>&1 || exit 1
$S --geo c5 --frames struct --variants fp32,fp32p,fp32xb,bf16,bf16_gradsoff,bf16_actoff --lrs 1e-4 --traj-variants fp32,bf16 > gpurun_out/r5b/study_c5_struct.txt 2>&1 || exit 1
$S --geo c4 --frames noise --variants fp32,fp32p,fp32xb,bf16,bf16_gradsoff,bf16_actoff --lrs 1e-5,1e-4 --traj-variants fp32,fp32xb,bf16 > gpurun_out/r5b/study_c4_noise.txt 2>&1 || exit 1
$S --geo c4 --frames struct --variants fp32,fp32p,fp32xb,bf16 --lrs 1e-4 --traj-variants fp32,bf16 > gpurun_out/r5b/study_c4_struct.txt 2>&1
