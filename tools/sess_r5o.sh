#!/bin/bash
# Round 5, session O: F(4×4,3×3) epilogue with one thread per (tile, channel pair) over 16-tile
# rounds (every point read once) vs the per-output-row threads (old): parity, stamps, decoder
# A/B at configs[1] / [4], library by library.
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_decoder.py tests/test_gpu_train_ops.py tests/test_gpu_configs.py -q -rfs -x --timeout 120 --timeout-method thread -k "f4x4 or wino or decoder or dual or config" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in old new; do
  SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,heads" --no-extras --reps 20 --stamps --xcd 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> $O/stamps.txt || exit 2
done
for rep in 1 2; do
  for v in old new; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 3
  done
done
for v in old new; do
  SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err || exit 4
done
