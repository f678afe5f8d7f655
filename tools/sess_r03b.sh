#!/bin/bash
# round-3 session: GPU suite, small-cin split A/B (conv_bench + decoder ab), bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03b
mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for s in 0 1 0 1; do
  SCFLOW_SMALLCIN_SPLIT=$s timeout -k 10 120 python tools/conv_bench.py --only "7x7,1->64" --no-extras > $OUT/cb_$s.txt 2>&1 || exit $?
  echo "split=$s"; cat $OUT/cb_$s.txt
done
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
head -c 400 $OUT/bench.json; echo
SCFLOW_SMALLCIN_SPLIT=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_s0.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_s1.json 2>&1 || exit $?
python3 -c "
import json
for t in ('s0','s1'):
    d=json.load(open('$OUT/bench_'+t+'.json')); print(t, d['value'], d['ms_per_step'])"
