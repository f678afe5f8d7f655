#!/bin/bash
# Round 5, session AM: pose-head FC K split (2 / 4 / 8 slices).
set -o pipefail
O=gpurun_out/r5am; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_bench.py --rounds 7 --steps 10 scflow_amd.modules.MultiClassPoseHead.fc_ksplit=2,4,8 > $O/ab.txt 2>&1 || exit 2
timeout -k 10 500 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 3 --steps 4 scflow_amd.modules.MultiClassPoseHead.fc_ksplit=4,8 > $O/ab_c4.txt 2>&1 || exit 3
