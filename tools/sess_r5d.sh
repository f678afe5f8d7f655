#!/bin/bash
# Round 5, session D: corr_net.0 variants in the decoder at configs[1] — wide 1x1 (default),
# conv1x1_kernel (SCFLOW_CONV1X1W=0), fused lookup + corr_net.0 (fuse_lookup_conv=1).
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O; export TMPDIR=/tmp
for w in 1 0; do
  SCFLOW_CONV1X1W=$w timeout -k 10 300 python -u tools/ab_bench.py --rounds 4 fuse_lookup_conv=0,1 2>&1 | grep -v amdgpu | sed "s/^/w$w /" >> $O/ab.txt || exit 5
done
