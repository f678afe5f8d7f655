#!/bin/bash
# round 4 session F: warp-specialised fused lookup + corr_net.0; Winograd U two sub-steps ahead
set -o pipefail
O=gpurun_out/r4f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py -k "fused or decoder or conv2d" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
SCFLOW_LIB=scflow_amd/lib/ab/uah2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv2d" > $O/pytest_uah2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_uah2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/lookup_conv_bench.py > $O/lc.txt 2>&1 || exit $?
timeout -k 10 180 python -u tools/lookup_conv_bench.py --batch 32 --size 64 --reps 20 >> $O/lc.txt 2>&1 || exit $?
for v in base uah2 base uah2; do
  L=""; [ $v != base ] && L=scflow_amd/lib/ab/$v.so
  SCFLOW_LIB=$L timeout -k 10 120 python tools/conv_bench.py --only "flow_net.1,out_net,mask_enc.1,dflow" --no-extras --reps 30 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/conv.txt || exit 3
  SCFLOW_LIB=$L timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> $O/ab.txt || exit 4
done
