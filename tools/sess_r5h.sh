#!/bin/bash
# Round 5, session H: bank-conflict-free Winograd halo pitches (true ds_read_b128 lane groups):
# parity of the Winograd convs, per-shape stamps old vs new library, decoder A/B.
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -q -rfs -x --timeout 120 --timeout-method thread -k "wino or gru or conv2d" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in old new; do
  SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 150 python -u tools/conv_bench.py --no-extras --reps 20 --stamps 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> $O/stamps.txt || exit 2
done
for rep in 1 2; do
  for v in old new; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 3
  done
done
