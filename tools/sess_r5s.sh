#!/bin/bash
# Round 5, session S: (1) the flow branch forked after the lookup + corr_net.0 launch
# (SCFLOW_FLOW_LATE / flow_branch_late); (2) output-channel blocks first for multi-round
# Winograd grids (SCFLOW_WINO_COFAST=1) at configs[4] — parity with each on, then A/Bs.
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O; export TMPDIR=/tmp
SCFLOW_FLOW_LATE=1 SCFLOW_WINO_COFAST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_configs.py tests/test_gpu_ops.py -q -rfs -x --timeout 120 --timeout-method thread -k "decoder or config or wino or gru" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 flow_branch_late=0,1 > $O/ab_flow_late.txt 2>&1 || exit 2
for v in 0 1; do
  SCFLOW_WINO_COFAST=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_cf$v.json 2> $O/bench_c4_cf$v.err || exit 3
done
for v in 0 1; do
  SCFLOW_WINO_COFAST=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_cf${v}_b.json 2> $O/bench_c4_cf${v}_b.err || exit 3
done
SCFLOW_WINO_COFAST=1 timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_c1_cf1.json 2> $O/bench_c1_cf1.err || exit 4
