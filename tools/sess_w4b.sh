#!/bin/bash
# F(4x4,3x3): phase stamps and the transform / GEMM split (kernel trace) on the decoder shapes.
set -o pipefail
O=gpurun_out/${1:-w4b}; mkdir -p $O; export TMPDIR=/tmp
R=$(pwd)
SCFLOW_CONV_WINO4=1 timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,out_net,heads" --no-extras --reps 20 --stamps 2>&1 | grep -v amdgpu > $O/stamps.txt || exit 2
cd /tmp
SCFLOW_CONV_WINO4=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run -- python3 $R/tools/conv_bench.py --only "corr_net.1,out_net,heads" --no-extras --reps 20 > /dev/null 2> $R/$O/kt.err || exit 3
DB=$(find $R/$O/kt -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "conv_bench wino4" > $R/$O/stats.txt
rm -rf $R/$O/kt
