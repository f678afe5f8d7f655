#!/bin/bash
# F(4x4,3x3) Winograd: parity (kernel tests; decoder / config tests with it on), conv_bench and
# decoder A/B against F(2x2,3x3).
set -o pipefail
O=gpurun_out/${1:-w4}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -rfs -x --timeout 120 --timeout-method thread -k "f4x4" > $O/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_k.log; [ $rc -eq 0 ] || exit $rc
SCFLOW_CONV_WINO4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_configs.py -q -rfs --timeout 200 --timeout-method thread > $O/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_dec.log; [ $rc -le 1 ] || exit $rc
for v in 0 1; do
  SCFLOW_CONV_WINO4=$v timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,out_net,heads,flow_net.1" --no-extras --reps 20 2>&1 | grep -v amdgpu | sed "s/^/w4=$v /" >> $O/conv.txt || exit 6
done
for rep in 1 2; do
  for v in 0 1; do
    SCFLOW_CONV_WINO4=$v timeout -k 10 300 python -u tools/ab_bench.py --rounds 2 2>&1 | grep -v amdgpu | sed "s/^/w4=$v /" >> $O/ab.txt || exit 5
  done
done
