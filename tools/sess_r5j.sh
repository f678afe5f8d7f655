#!/bin/bash
# Round 5, session J: tile-row lookup with two level regions per pixel slot (6 workgroups per CU
# instead of 4): parity of the lookups, configs[4] lookup alone (stamps) and the decoder at
# configs[4] / configs[1], previous library (new) vs this one (tb2).
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_library.py tests/test_gpu_configs.py -q -rfs -x --timeout 120 --timeout-method thread -k "tiled or lookup or config4" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for v in new tb2; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps $([ $rep = 1 ] && echo --check) 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/lookup.txt || exit 3
  done
done
for rep in 1 2; do
  for v in new tb2; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_${v}_$rep.json 2> $O/bench_c4_${v}_$rep.err || exit 4
  done
done
