#!/bin/bash
# Round 5, session K: paired F(4,5) workgroups (SCFLOW_WINO5_PAIR=1: two tile blocks per 512-thread
# workgroup, meeting at every barrier) — parity with it on, GRU stamps, decoder A/B at configs[1]
# and configs[4]; ping-pong halves and hipGraph replay re-measured on the current kernel set.
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O; export TMPDIR=/tmp
SCFLOW_WINO5_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_configs.py -q -rfs -x --timeout 120 --timeout-method thread -k "gru or conv2d or decoder or config1 or config4" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCFLOW_WINO5_PAIR=$v timeout -k 10 150 python -u tools/conv_bench.py --no-extras --reps 20 --stamps --xcd --only "gru" 2>&1 | grep -v amdgpu | sed "s/^/pair=$v /" >> $O/stamps.txt || exit 2
done
for rep in 1 2; do
  for v in 0 1; do
    SCFLOW_WINO5_PAIR=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_p${v}_$rep.json 2> $O/bench_p${v}_$rep.err || exit 3
  done
done
for v in 0 1; do
  SCFLOW_WINO5_PAIR=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_p$v.json 2> $O/bench_c4_p$v.err || exit 4
done
timeout -k 10 300 python -u tools/ab_bench.py --rounds 3 --steps 10 pingpong=0,1 > $O/ab_pingpong.txt 2>&1 || exit 5
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --graph > $O/bench_graph.json 2> $O/bench_graph.err || exit 6
