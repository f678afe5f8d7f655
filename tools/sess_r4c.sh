#!/bin/bash
# round 4 session C: GPU tests of this round's changes; wide 1x1 and fused lookup+corr_net.0 A/B
# (configs[1] and configs[4]); training timing with / without gc.freeze
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_library.py tests/test_gpu_render.py tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_train_ops.py tests/test_gpu_train.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
[ $rc -le 1 ] || exit $rc  # test failures: go on measuring; a crash / time limit: stop here
SCFLOW_CONV1X1W=0 timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 fuse_lookup_conv=0 > $O/ab_old.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 fuse_lookup_conv=0,1 > $O/ab_new.txt 2>&1 || exit $?
SCFLOW_CONV1X1W=0 timeout -k 10 300 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 3 --steps 3 fuse_lookup_conv=0 > $O/ab512_old.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 3 --steps 3 fuse_lookup_conv=0,1 > $O/ab512_new.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/train_timing.py --steps 20 > $O/tt.json 2> $O/tt.err &&
timeout -k 10 300 python -u tools/train_timing.py --steps 20 --freeze > $O/tt_freeze.json 2> $O/tt_freeze.err
