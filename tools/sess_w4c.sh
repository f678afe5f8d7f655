#!/bin/bash
# F(4x4,3x3): parity, phase stamps, transform/GEMM split, decoder A/B.
set -o pipefail
O=gpurun_out/${1:-w4c}; mkdir -p $O; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -rfs -x --timeout 120 --timeout-method thread -k "f4x4" > $O/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_k.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCFLOW_CONV_WINO4=$v timeout -k 10 120 python -u tools/conv_bench.py --only "corr_net.1,out_net,heads" --no-extras --reps 20 --stamps 2>&1 | grep -v amdgpu | sed "s/^/w4=$v /" >> $O/stamps.txt || exit 2
done
cd /tmp
SCFLOW_CONV_WINO4=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run -- python3 $R/tools/conv_bench.py --only "corr_net.1,out_net,heads" --no-extras --reps 20 > /dev/null 2> $R/$O/kt.err || exit 3
DB=$(find $R/$O/kt -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "conv_bench wino4" > $R/$O/stats.txt
python3 $R/tools/kern_durations.py $DB wino4 > $R/$O/durations.txt
rm -rf $R/$O/kt
cd $R
for rep in 1 2; do
  for v in 0 1; do
    SCFLOW_CONV_WINO4=$v timeout -k 10 300 python -u tools/ab_bench.py --rounds 2 2>&1 | grep -v amdgpu | sed "s/^/w4=$v /" >> $O/ab.txt || exit 5
  done
done
