#!/bin/bash
# Round 5, session AH: automatic stream priority (high-priority critical stream above 32² maps):
# decoder / refiner / library GPU tests, the configs[4] and configs[1] bench lines.
set -o pipefail
O=gpurun_out/r5ah; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_encoder.py tests/test_gpu_library.py tests/test_gpu_render.py -m gpu > $O/test.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 3
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_c1.json 2> $O/bench_c1.err || exit 4
