#!/bin/bash
# Round 5, session Z: small-cin MFMA conv with the bias prefetched and a branch-free store loop.
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "flow_net.0,mask_enc.0" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 env:SCFLOW_SMALLCIN_SPLIT=0,1 > $O/ab.txt 2>&1 || exit 4
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 4 --steps 5 > $O/ab_c4.txt 2>&1 || exit 5
