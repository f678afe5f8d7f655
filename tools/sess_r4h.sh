#!/bin/bash
# Decoder A/B of round 4's opt-in paths: K splits x fused lookup + corr_net.0 (configs[1]), the
# fused kernel at configs[4]; standalone lookup / conv timings
set -o pipefail
O=gpurun_out/r4h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lookup_conv_bench.py > $O/lc.txt 2>&1 || exit $?
timeout -k 10 180 python -u tools/lookup_conv_bench.py --batch 32 --size 64 --reps 20 >> $O/lc.txt 2>&1 || exit $?
for ks in 1 0; do
  SCFLOW_WINO_KSPLIT=$ks SCFLOW_WINO5_KSPLIT=$ks timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/ks$ks /" >> $O/ab.txt || exit 5
done
timeout -k 10 300 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 2 --steps 3 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/c4 /" >> $O/ab.txt || exit 7
