#!/bin/bash
# round-4 evidence at HEAD: the GPU suite, the bench line (configs[1]) and the configs[4] line,
# kernel-trace + PMC traffic profiles (tools/prof_session.sh), the training-step kernel stats
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_$TAG; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
head -c 300 $OUT/bench.json; echo
timeout -k 10 400 python bench.py --batch 32 --size 512 --iters 12 --steps 5 --warmup 2 --e2e-batch 0 --train-batch 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
head -c 300 $OUT/bench_c4.json; echo
bash tools/prof_session.sh $TAG || exit $?
cd /tmp
B4="--batch 32 --size 512 --iters 12 --steps 3 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt4 -o run -- python3 $R/bench.py $B4 > $OUT/bench_kt4.json 2> $OUT/kt4.err || exit $?
DB=$(find $OUT/kt4 -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python bench.py $B4" > $OUT/stats_c4.txt
python3 $R/tools/prof_summary.py $DB 8 > $OUT/per_forward_c4.txt  # 1 warmup + 3 timed + 1 + 3 secondary-timer forwards
rm -rf $OUT/kt4
cd $R && bash tools/train_prof.sh > $OUT/train_prof.log 2>&1 || exit $?
