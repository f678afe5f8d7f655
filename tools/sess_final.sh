#!/bin/bash
# round-end evidence at HEAD: the GPU suite, the full bench line, kernel-trace + PMC traffic profiles
TAG=${1:-r03f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_$TAG; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
head -c 300 $OUT/bench.json; echo
bash tools/prof_session.sh $TAG || exit $?
