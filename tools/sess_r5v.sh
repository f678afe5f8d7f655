#!/bin/bash
# Round 5, session V: F(4×4,3×3) GEMM depth, in-process interleaved A/B (auto vs one in flight).
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 env:SCFLOW_WINO4_DEPTH=0,1 > $O/ab_depth.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 5 --steps 5 env:SCFLOW_WINO4_DEPTH=0,1 > $O/ab_depth_c4.txt 2>&1 || exit 3
