#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
# Stops at the first step that faults / aborts / times out (rc other than 0 or 1 for pytest).
# usage: tools/gpu_session.sh [tag] [what: all|test|bench|prof]
TAG=${1:-r01}
WHAT=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

if [ $WHAT = all ] || [ $WHAT = test ]; then
  timeout -k 10 600 python -m pytest $R/tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a $OUT/pytest_gpu_$TAG.log
  ok $rc || exit $rc
fi
if [ $WHAT = all ] || [ $WHAT = bench ]; then
  timeout -k 10 400 python $R/bench.py --steps 10 --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ $WHAT = all ] || [ $WHAT = prof ]; then
  cd /tmp
  # decoder-only (the bench's roofline kernel averages must agree with this profile)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- \
      python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  # end-to-end refiner (configs[2]) kernels
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_e2e_$TAG -o run -- \
      python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 3 --train-batch 0 > $OUT/bench_prof_e2e_$TAG.json 2> $OUT/prof_e2e_$TAG.err
  rc=$?; echo "rocprof e2e rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  find $OUT/prof_$TAG -name "*stats*" | head
fi
if [ $WHAT = all ] || [ $WHAT = prof ] || [ $WHAT = trainprof ]; then
  cd /tmp
  # training step (configs[3] per GPU)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_train_$TAG -o run -- \
      python $R/tools/train_bench.py --steps 3 --warmup 2 > $OUT/bench_prof_train_$TAG.json 2> $OUT/prof_train_$TAG.err
  rc=$?; echo "rocprof train rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  db=$(find $OUT/prof_train_$TAG -name "*.db" | head -1)
  python $R/tools/stats_file.py $db "python tools/train_bench.py --steps 3 --warmup 2 (5 training steps, B=16, 256x256, 8 iters)" > $OUT/train_stats_$TAG.txt
  python $R/tools/busy.py $db > $OUT/train_busy_$TAG.txt 2>&1 || true
  rm -rf $OUT/prof_train_$TAG
fi
