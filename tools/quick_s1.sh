# quick GPU check: targeted tests + training-step timing + per-shape conv/wgrad/gemm timing
set -o pipefail
T=${TAG:-s1}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread tests/test_gpu_train_ops.py ${TESTS:-} > gpurun_out/$T/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/$T/tests.log; exit 1; }
grep "wino5 wgrad" gpurun_out/$T/tests.log | tail -2 || true
tail -1 gpurun_out/$T/tests.log
timeout -k 10 200 python tools/train_bench.py --steps 5 --warmup 3 > gpurun_out/$T/train.txt 2>&1 || exit 1
timeout -k 10 250 python tools/dbg/train_conv_shapes.py > gpurun_out/$T/shapes_conv.txt 2>&1 || exit 1
tail -1 gpurun_out/$T/train.txt
