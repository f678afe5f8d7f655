#!/bin/bash
# round 4 session D: why the wide 1x1 / fused kernels lose in the decoder — standalone timings and
# an in-decoder kernel trace; library tests again
set -o pipefail
O=gpurun_out/r4d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_library.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/lookup_conv_bench.py > $O/lc.txt 2>&1 || exit $?
timeout -k 10 180 python -u tools/lookup_conv_bench.py --batch 32 --size 64 --reps 20 >> $O/lc.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/ab_bench.py --rounds 1 --steps 5 fuse_lookup_conv=1 > $O/prof.log 2>&1 || exit $?
