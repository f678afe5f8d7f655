#!/bin/bash
# Round 5, session N: F(4×4,3×3) point GEMM with 6 column-owning waves (conv_wino4c_kernel,
# SCFLOW_WINO4_COL=1) vs the 4-wave kernel (0): parity, stamps, decoder A/B at configs[1] / [4].
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_train_ops.py -q -rfs -x --timeout 120 --timeout-method thread -k "f4x4 or wino or decoder or dual" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCFLOW_WINO4_COL=$v timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,heads" --no-extras --reps 20 --stamps --xcd 2>&1 | grep -v amdgpu | sed "s/^/col=$v /" >> $O/stamps.txt || exit 2
done
for rep in 1 2; do
  for v in 0 1; do
    SCFLOW_WINO4_COL=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_col${v}_$rep.json 2> $O/bench_col${v}_$rep.err || exit 3
  done
done
for v in 0 1; do
  SCFLOW_WINO4_COL=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_col$v.json 2> $O/bench_c4_col$v.err || exit 4
done
