#!/bin/bash
# round 4 session B: new GPU tests (torch.library ops, GRU shared weights, dX shortcuts, training
# parity, renderer light wiring) + training-step GC instrumentation with / without gc.freeze
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_library.py tests/test_gpu_render.py tests/test_gpu_train_ops.py tests/test_gpu_train.py > gpurun_out/r4b/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/train_timing.py --steps 20 > gpurun_out/r4b/tt.json 2> gpurun_out/r4b/tt.err &&
timeout -k 10 300 python -u tools/train_timing.py --steps 20 --freeze > gpurun_out/r4b/tt_freeze.json 2> gpurun_out/r4b/tt_freeze.err
