#!/bin/bash
# Round 5, session X: small-cin MFMA conv with every global load in flight before the halo stores.
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --only "flow_net.0,mask_enc.0" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --batch 32 --size 64 --only "flow_net.0,mask_enc.0" > $O/conv_c4.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 4
