#!/bin/bash
# Round 5, session L: the deferred full-resolution pose-step launches after corr_net.1 (beside
# out_net / the GRU) instead of right after the flow branch — parity with it on, decoder A/B.
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O; export TMPDIR=/tmp
SCFLOW_FULLRES_LATE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_configs.py tests/test_gpu_graph.py -q -rfs -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 fullres_late=0,1 > $O/ab_c1.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 2 --steps 4 fullres_late=0,1 > $O/ab_c4.txt 2>&1 || exit 3
SCFLOW_FULLRES_LATE=1 timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_late.json 2> $O/bench_late.err || exit 4
