#!/bin/bash
# Round 5, session AA: F(4×4,3×3) GEMM with the epilogue's per-channel operands fetched up front.
set -o pipefail
O=gpurun_out/r5aa; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "f4x4" > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "corr_net.1,heads" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 4
