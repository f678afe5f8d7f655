#!/bin/bash
# round 4 session A: training-step host/GPU split, configs[4] bench line, default bench
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u tools/train_timing.py --steps 12 > gpurun_out/r4a/train_timing.json 2> gpurun_out/r4a/train_timing.err &&
timeout -k 10 240 python -u tools/train_timing.py --steps 12 --graph > gpurun_out/r4a/train_timing_graph.json 2> gpurun_out/r4a/train_timing_graph.err &&
timeout -k 10 300 python -u bench.py --batch 32 --size 512 --iters 12 --e2e-batch 0 --train-batch 0 --no-cpu-baseline > gpurun_out/r4a/bench_c4.json 2> gpurun_out/r4a/bench_c4.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err
