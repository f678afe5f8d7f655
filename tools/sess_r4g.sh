#!/bin/bash
# round 4 session G: tests of this round's kernels (fused lookup + corr_net.0, K-split 32-channel
# Winograd, static wgrad pipelines, residual-gradient hand-over); Winograd phase stamps; wgrad
# shapes and training step A/B
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py -k "fused or decoder or conv2d" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py tests/test_gpu_train.py -k "wgrad or conv2d_nhwc or configs3 or batch_norm or instance_norm or dual or relu_mask" > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_train.log; [ $rc -le 1 ] || exit $rc
for ks in 1 0; do
  SCFLOW_WINO_KSPLIT=$ks SCFLOW_WINO5_KSPLIT=$ks timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,flow_net.1,out_net,heads,dflow.1,mask_enc.1,gru" --no-extras --reps 20 --stamps 2>&1 | sed "s/^/ks$ks /" >> $O/stamps.txt || exit 6
done
for v in base ww0; do
  L=""; [ $v != base ] && L=scflow_amd/lib/ab/$v.so
  SCFLOW_LIB=$L timeout -k 10 200 python -u tools/wgrad_bench.py --reps 10 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/wgrad.txt || exit 3
done
for v in base ww0 fuse0; do
  L=""; E=1; [ $v = ww0 ] && L=scflow_amd/lib/ab/$v.so; [ $v = fuse0 ] && E=0
  SCFLOW_TRAIN_BN_FUSED=$E SCFLOW_TRAIN_RES_GRAD=$E SCFLOW_TRAIN_HEADS_FUSED=$E SCFLOW_TRAIN_RELU_MASK=$E SCFLOW_LIB=$L timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt_$v.json 2> $O/tt_$v.err || exit 4
  echo "$v $(cat $O/tt_$v.json | head -c 400)" >> $O/tt.txt
done
