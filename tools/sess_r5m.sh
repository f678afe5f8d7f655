#!/bin/bash
# Round 5, session M: the pose head's heads inside the pose step's launch (scflow_pose_step_heads)
# — its parity test, the decoder / pose-head / config tests, decoder A/B at configs[1] / [4].
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_encoder.py -q -rfs -x --timeout 120 --timeout-method thread -k "pose or decoder or config or graph or refiner" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 fuse_heads=0,1 > $O/ab_c1.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 2 --steps 4 fuse_heads=0,1 > $O/ab_c4.txt 2>&1 || exit 3
# F(4×4,3×3) also for every conv whose GEMM grid fills the chip twice (SCFLOW_CONV_WINO4=3) vs
# cout ≥ 160 only (1) vs every eligible conv (2): configs[4] and configs[1]
for v in 1 3 2; do
  SCFLOW_CONV_WINO4=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_w$v.json 2> $O/bench_c4_w$v.err || exit 4
done
for v in 1 2; do
  SCFLOW_CONV_WINO4=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_c1_w$v.json 2> $O/bench_c1_w$v.err || exit 5
done
