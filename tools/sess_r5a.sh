#!/bin/bash
# Round 5, session A: the whole default GPU suite at HEAD (no -x: every collected test is
# reached), then the opt-in suite with every round-4 switch on and the static-wgrad library,
# then the round-4 A/Bs (as in tools/sess_r4g.sh, tools/sess_r4h.sh).  Build on the CPU first:
#   python -m scflow_amd.build && tools/build_variant.sh ws1 train.hip "-DWW_STATIC=1 -DW5W_STATIC=1"
set -o pipefail
O=gpurun_out/r5a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfs --timeout 120 --timeout-method thread > $O/pytest_default.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_default.log; [ $rc -le 1 ] || exit $rc
WS=scflow_amd/lib/ab/ws1.so
ON="SCFLOW_TEST_OPTIN=1 SCFLOW_WINO_KSPLIT=1 SCFLOW_WINO5_KSPLIT=1 SCFLOW_TRAIN_BN_FUSED=1 SCFLOW_TRAIN_RELU_MASK=1 SCFLOW_TRAIN_HEADS_FUSED=1 SCFLOW_TRAIN_RES_GRAD=1"
env $ON SCFLOW_LIB=$WS timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfs --timeout 200 --timeout-method thread > $O/pytest_optin.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_optin.log; [ $rc -le 1 ] || exit $rc
# K split on / off: Winograd phase stamps of the decoder shapes
for ks in 1 0; do
  SCFLOW_WINO_KSPLIT=$ks SCFLOW_WINO5_KSPLIT=$ks timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,flow_net.1,out_net,heads,dflow.1,mask_enc.1,gru" --no-extras --reps 20 --stamps 2>&1 | sed "s/^/ks$ks /" >> $O/stamps.txt || exit 6
done
# static-pipeline weight gradients vs the loop ones
for v in base ws1; do
  L=""; [ $v != base ] && L=$WS
  SCFLOW_LIB=$L timeout -k 10 200 python -u tools/wgrad_bench.py --reps 10 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/wgrad.txt || exit 3
done
# decoder: K splits x fused lookup + corr_net.0 at configs[1], the fused kernel at configs[4]
for ks in 1 0; do
  SCFLOW_WINO_KSPLIT=$ks SCFLOW_WINO5_KSPLIT=$ks timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/ks$ks /" >> $O/ab.txt || exit 5
done
timeout -k 10 300 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 2 --steps 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/c4 /" >> $O/ab.txt || exit 7
# training step: base, static wgrads, every switch
for v in base ws1 all; do
  L=""; E=0; [ $v != base ] && L=$WS; [ $v = all ] && E=1
  SCFLOW_TRAIN_BN_FUSED=$E SCFLOW_TRAIN_RES_GRAD=$E SCFLOW_TRAIN_HEADS_FUSED=$E SCFLOW_TRAIN_RELU_MASK=$E SCFLOW_WINO_KSPLIT=$E SCFLOW_WINO5_KSPLIT=$E SCFLOW_LIB=$L timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt_$v.json 2> $O/tt_$v.err || exit 4
  echo "$v $(head -c 400 $O/tt_$v.json)" >> $O/tt.txt
done
