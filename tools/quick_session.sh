#!/bin/bash
# Iteration loop on the GPU box: a pytest subset, the decoder bench leg, a kernel trace with the
# per-forward table and one iteration's timeline.
# usage: tools/quick_session.sh TAG "PYTEST -k EXPR" [extra bench args]
TAG=${1:-q}
K=${2:-"pose or decoder"}
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/q_$TAG
mkdir -p $OUT
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 5 ] || exit $rc
B="--steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 $@"
timeout -k 10 300 python bench.py $B > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py $B > /dev/null 2> $OUT/kt.err || exit $?
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/prof_summary.py $DB 24 > $OUT/per_forward.txt
python3 $R/tools/timeline.py $DB --iteration 61 > $OUT/timeline.txt 2>&1
rm -rf $OUT/kt
head -16 $OUT/per_forward.txt; tail -1 $OUT/timeline.txt
