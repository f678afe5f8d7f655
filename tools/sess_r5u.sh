#!/bin/bash
# Round 5, session U: F(4×4,3×3) GEMM with two sub-steps of V / U in flight (one workgroup per
# CU) vs one: parity, then the two update-block shapes alone with stamps, then the decoder.
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "f4x4" > $O/test.txt 2>&1 || exit 2
for d in 1 2; do
  SCFLOW_WINO4_DEPTH=$d timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "corr_net.1,heads,out_net" > $O/conv_d$d.txt 2>&1 || exit 3
done
for d in 1 2 0; do
  SCFLOW_WINO4_DEPTH=$d timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 > $O/ab_d$d.txt 2>&1 || exit 4
done
