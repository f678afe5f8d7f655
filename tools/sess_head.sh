#!/bin/bash
# HEAD evidence in one call: the whole GPU suite (no -x, every collected test reached), smoke,
# the default bench line, the configs[4] bench line, then tools/prof_r5.sh (kernel traces,
# timeline, PMC traffic/SQ passes).  usage: tools/sess_head.sh TAG → gpurun_out/head_TAG/
TAG=${1:-r5h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/head_$TAG; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit 5
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 6
head -c 300 $OUT/bench.json; echo
timeout -k 10 300 python bench.py --batch 32 --size 512 --iters 12 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 7
head -c 300 $OUT/bench_c4.json; echo
[ -n "$NOPROF" ] && exit 0
bash tools/prof_r5.sh $TAG || exit $?
