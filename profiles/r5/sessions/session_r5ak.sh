# kernel trace: the fp32 1x1/2 downsample dgrad, per-class launches vs one launch
set -o pipefail
R=$PWD
O=$R/gpurun_out/s5ak; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/cl -o run -- \
  python3 $R/scripts/convbench.py --frames 640 --reps 2 --wt32 --bnbwd --kinds dgrad --only 256:512:1:56,128:128:3:56 --classes > $O/cl.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/par -o run -- \
  python3 $R/scripts/convbench.py --frames 640 --reps 2 --wt32 --bnbwd --kinds dgrad --only 256:512:1:56,128:128:3:56 > $O/par.log 2>&1
