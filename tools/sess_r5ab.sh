#!/bin/bash
# Round 5, session AB: pose-head K-split targets (conv1/conv2 MFMA halo conv, conv3 gather conv).
set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_bench.py --rounds 5 --steps 10 scflow_amd.modules.MultiClassPoseHead.conv_wg_target=256,512,1024 scflow_amd.modules.MultiClassPoseHead.gather_wg_target=64,128,256 > $O/ab.txt 2>&1 || exit 2
timeout -k 10 500 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 3 --steps 4 scflow_amd.modules.MultiClassPoseHead.conv_wg_target=256,512,1024 > $O/ab_c4.txt 2>&1 || exit 3
