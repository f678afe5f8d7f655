#!/bin/bash
# Lookup A/B at configs[4]: tiled b32 regions (SCFLOW_LK_TB=0) vs tile-row regions (1); parity first.
set -o pipefail
O=gpurun_out/${1:-lk5}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_library.py -q -rfs --timeout 120 --timeout-method thread -k "tiled or lookup" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for tb in 0 1; do
    SCFLOW_LK_TB=$tb timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps $([ $rep = 1 ] && echo --check) 2>&1 | grep -v amdgpu.ids | sed "s/^/tb$tb /" >> $O/lookup.txt || exit 3
  done
done
SCFLOW_LK_TB=1 timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps --batch 16 --size 256 2>&1 | grep -v amdgpu.ids | sed "s/^/c1 /" >> $O/lookup.txt || exit 3
