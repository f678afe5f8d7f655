#!/bin/bash
# GroupNorm reduce in 16-channel blocks (twice the workgroups) vs 32: parity, the pose head's
# kernels alone, in-process decoder A/B at configs[1] and configs[4].
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5at; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "pose or decoder or config or refine or group_norm or gn" > $OUT/test.txt 2>&1
rc=$?; tail -2 $OUT/test.txt; [ $rc -eq 0 ] || exit $rc
for v in 16 32; do SCFLOW_GNR_CB=$v timeout -k 10 200 python tools/ph_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/cb$v /" || exit 3; done > $OUT/ph.txt
cat $OUT/ph.txt
timeout -k 10 300 python tools/ab_bench.py --rounds 7 env:SCFLOW_GNR_CB=16,32 > $OUT/ab.txt 2>&1 || exit 4
cat $OUT/ab.txt
timeout -k 10 300 python tools/ab_bench.py --rounds 5 --batch 32 --size 512 --iters 12 env:SCFLOW_GNR_CB=16,32 > $OUT/ab_c4.txt 2>&1 || exit 5
cat $OUT/ab_c4.txt
