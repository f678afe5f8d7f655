#!/bin/bash
# Round 5, session AC: F(4,5) q kernels with the epilogue's global reads issued as the main loop starts.
set -o pipefail
O=gpurun_out/${OUTDIR:-r5ac}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/conv_bench.py --no-extras --stamps --only "gru" > $O/conv.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 4
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 4 --steps 5 > $O/ab_c4.txt 2>&1 || exit 5
