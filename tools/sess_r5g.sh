#!/bin/bash
# Round 5, session G: bench line with the GRU (conv_wino5_kernel) headline, then the HEAD
# evidence pass (kernel traces, FETCH/WRITE/SQ PMC at configs[1] and configs[4]).
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 5
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 6
bash tools/prof_r5.sh r5g > $O/prof.log 2>&1 || exit 7
