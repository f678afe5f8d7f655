#!/bin/bash
# Round 5, session Q: workgroups per image of the deferred full-resolution pose step (it runs on
# the side stream beside the correlation branch; fewer workgroups = a lower, longer bandwidth
# draw), SCFLOW_FULLRES_BLOCKS = 8 / 16 / 32 / 64 (default).
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for v in 64 32 16 8; do
    SCFLOW_FULLRES_BLOCKS=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_fb${v}_$rep.json 2> $O/bench_fb${v}_$rep.err || exit 3
  done
done
for v in 64 16; do
  SCFLOW_FULLRES_BLOCKS=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_fb$v.json 2> $O/bench_c4_fb$v.err || exit 4
done
# the flow branch forked after the lookup + corr_net.0 launch (beside corr_net.1)
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 flow_branch_late=0,1 > $O/ab_flow_late.txt 2>&1 || exit 5
SCFLOW_FLOW_LATE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_configs.py -q -x --timeout 120 --timeout-method thread -k "decoder or config1" > $O/pytest_flow_late.log 2>&1 || exit 6
