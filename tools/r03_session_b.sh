#!/bin/bash
# round-3 session: STREAM ceiling + counter calibration, the configs[3] shard test, bench, profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/micro/stream_session.sh r03 || exit $?
SCFLOW_TRAIN_ERRS=gpurun_out/train_errs_c3.json timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v --timeout 600 --timeout-method thread -p no:cacheprovider -k configs3 > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/prof_session.sh r03b
