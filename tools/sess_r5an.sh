#!/bin/bash
# Round 5, session AN: F(2×2,3×3) epilogue with the per-channel operands fetched up front and the
# activation a constant of the store loop.
set -o pipefail
O=gpurun_out/r5an; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_encoder.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "out_net,flow_net.1,dflow.1,mask_enc.1" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 4
