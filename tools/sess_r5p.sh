#!/bin/bash
# Round 5, session P: HEAD evidence — the whole GPU suite, the default bench line (with e2e,
# training, CPU baseline), then tools/prof_r5.sh (kernel traces, timeline, FETCH/WRITE/SQ PMC at
# configs[1] and configs[4], traffic JSONs).
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfs -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 5
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 6
bash tools/prof_r5.sh r5p > $O/prof.log 2>&1 || exit 7
