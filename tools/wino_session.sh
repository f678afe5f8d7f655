#!/bin/bash
# Winograd conv check: parity tests, then isolated conv timings with and without Winograd.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-w1}
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -x -q -p no:cacheprovider -k "conv" \
  --timeout 120 --timeout-method thread > $OUT/wino_pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/wino_pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python $R/tools/conv_bench.py --batch 16 > $OUT/wino_convbench_$TAG.txt 2>&1 || exit $?
SCFLOW_CONV_WINO=0 timeout -k 10 200 python $R/tools/conv_bench.py --batch 16 > $OUT/direct_convbench_$TAG.txt 2>&1 || exit $?
paste -d'|' $OUT/direct_convbench_$TAG.txt $OUT/wino_convbench_$TAG.txt
