#!/bin/bash
# Round 5, session AI: whole-halo thin predictor on 64-wide maps (32-column tiles).
set -o pipefail
O=gpurun_out/r5ai; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_train_ops.py -m gpu > $O/test.txt 2>&1 || exit 2
for v in 1 0; do
  SCFLOW_THIN_FULL=$v timeout -k 10 120 python -u tools/conv_bench.py --no-extras --batch 32 --size 64 --only "flow_pred" > $O/conv_full$v.txt 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 4
SCFLOW_THIN_FULL=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_off.json 2> $O/bench_c4_off.err || exit 5
