#!/bin/bash
# Round 5, session AJ: chunked thin predictors with an XCD-aware tile order.
set -o pipefail
O=gpurun_out/r5aj; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --batch 32 --size 64 --only "flow_pred,mask_pred" > $O/conv_c4.txt 2>&1 || exit 3
SCFLOW_THIN_FULL=0 timeout -k 10 120 python -u tools/conv_bench.py --no-extras --only "flow_pred,mask_pred" > $O/conv_c1_chunked.txt 2>&1 || exit 3
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --only "flow_pred,mask_pred" > $O/conv_c1.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 4
