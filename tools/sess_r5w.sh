#!/bin/bash
# Round 5, session W: thin predictors with lanes over channels vs the LDS-staged kernels.
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "thin or variants" > $O/test.txt 2>&1 || exit 2
for v in 0 1; do
  SCFLOW_THIN_LANE=$v timeout -k 10 120 python -u tools/conv_bench.py --no-extras --only "flow_pred,mask_pred" > $O/conv_lane$v.txt 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 env:SCFLOW_THIN_LANE=1,0 > $O/ab_lane.txt 2>&1 || exit 4
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 4 --steps 5 env:SCFLOW_THIN_LANE=1,0 > $O/ab_lane_c4.txt 2>&1 || exit 5
