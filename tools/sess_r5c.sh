#!/bin/bash
# Round 5, session C: the whole GPU suite after the opt-in promotions / removals.
set -o pipefail
O=gpurun_out/r5c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfs --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt.json 2> $O/tt.err || exit 4
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 5
