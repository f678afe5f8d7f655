#!/bin/bash
# Round 5, session F: F(4x4,3x3) on by default (cout >= 160): whole GPU suite, bench line, training step.
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfs --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 5
for v in 1 0; do
  SCFLOW_CONV_WINO4=$v timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt_w$v.json 2> $O/tt_w$v.err || exit 4
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 6
