#!/bin/bash
# Round 5, session AG: the forward's critical stream at high priority vs the caller's stream.
set -o pipefail
O=gpurun_out/r5ag2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 main_priority=0,1,2 > $O/ab.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 4 --steps 5 main_priority=0,1,2 > $O/ab_c4.txt 2>&1 || exit 3
