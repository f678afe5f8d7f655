#!/bin/bash
# round 4 session E: the wide 1x1 / fused kernels after the straight-line rewrite; Winograd
# U-reload scheduling barriers (default: 32-channel F(2x2,3x3) workgroups + F(4,5); variants: none,
# every workgroup width)
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_library.py tests/test_gpu_ops.py -k "library or conv2d or fused or pick_bk or opcheck or registered or compile or modules or gru" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/lookup_conv_bench.py > $O/lc.txt 2>&1 || exit $?
timeout -k 10 180 python -u tools/lookup_conv_bench.py --batch 32 --size 64 --reps 20 >> $O/lc.txt 2>&1 || exit $?
for v in base nosb sball base; do
  L=""; [ $v != base ] && L=scflow_amd/lib/ab/$v.so
  SCFLOW_LIB=$L timeout -k 10 120 python tools/conv_bench.py --only "flow_net.1,out_net,mask_enc.1,heads,corr_net.1,gru" --no-extras --reps 30 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/conv.txt || exit 3
  SCFLOW_LIB=$L timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> $O/ab.txt || exit 4
done
SCFLOW_CONV1X1W=0 timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 fuse_lookup_conv=0 2>&1 | grep -v amdgpu | sed "s/^/old1x1 /" >> $O/ab.txt || exit 5
