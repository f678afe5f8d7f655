#!/bin/bash
# Validation + A/B of round 4's opt-in paths.  Build the static-wgrad variant on
# the CPU first:  tools/build_variant.sh ws1 train.hip "-DWW_STATIC=1 -DW5W_STATIC=1"
# Then: the opt-in GPU tests with every switch on (and the static-wgrad library), Winograd phase
# stamps with / without the K splits, the wgrad shapes and the training step with / without.
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O; export TMPDIR=/tmp
WS=scflow_amd/lib/ab/ws1.so
ON="SCFLOW_TEST_OPTIN=1 SCFLOW_WINO_KSPLIT=1 SCFLOW_WINO5_KSPLIT=1 SCFLOW_TRAIN_BN_FUSED=1 SCFLOW_TRAIN_RELU_MASK=1 SCFLOW_TRAIN_HEADS_FUSED=1 SCFLOW_TRAIN_RES_GRAD=1"
env $ON timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_decoder.py -k "fused or decoder or conv2d" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
env $ON SCFLOW_LIB=$WS timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py tests/test_gpu_train.py -k "wgrad or conv2d_nhwc or configs3 or batch_norm or instance_norm or dual or relu_mask" > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_train.log; [ $rc -le 1 ] || exit $rc
for ks in 1 0; do
  SCFLOW_WINO_KSPLIT=$ks SCFLOW_WINO5_KSPLIT=$ks timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,flow_net.1,out_net,heads,dflow.1,mask_enc.1,gru" --no-extras --reps 20 --stamps 2>&1 | sed "s/^/ks$ks /" >> $O/stamps.txt || exit 6
done
for v in base ws1; do
  L=""; [ $v != base ] && L=$WS
  SCFLOW_LIB=$L timeout -k 10 200 python -u tools/wgrad_bench.py --reps 10 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/wgrad.txt || exit 3
done
for v in base ws1 all; do
  L=""; E=0; [ $v != base ] && L=$WS; [ $v = all ] && E=1
  SCFLOW_TRAIN_BN_FUSED=$E SCFLOW_TRAIN_RES_GRAD=$E SCFLOW_TRAIN_HEADS_FUSED=$E SCFLOW_TRAIN_RELU_MASK=$E SCFLOW_WINO_KSPLIT=$E SCFLOW_WINO5_KSPLIT=$E SCFLOW_LIB=$L timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt_$v.json 2> $O/tt_$v.err || exit 4
  echo "$v $(cat $O/tt_$v.json | head -c 400)" >> $O/tt.txt
done
