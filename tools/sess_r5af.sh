#!/bin/bash
# Round 5, session AF: whole-halo thin predictor with its weights in LDS (workgroup stamps, parity,
# decoder).
set -o pipefail
O=gpurun_out/r5af2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "flow_pred" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 4
