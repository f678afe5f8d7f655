#!/bin/bash
# Round 5, final HEAD validation: the whole GPU suite, smoke(), the default bench line (with e2e,
# training, CPU baseline) and the configs[4] line.  The kernel evidence of the same tree is
# session R (tools/prof_r5.sh r, run after these steps).
set -o pipefail
O=gpurun_out/r5fin2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfs -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 5
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4.json 2> $O/bench_c4.err || exit 6
bash tools/prof_r5.sh r > $O/prof.log 2>&1 || exit 7
