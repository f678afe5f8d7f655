# Training-step profile (configs[3], B=16): eager and graph step times, then a rocprofv3 kernel
# trace of eager (default) or graph (MODE=graph) steps -> per-kernel stats, busy/idle breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trainprof
MODE=${MODE:-eager}
GFLAG=""
[ "$MODE" = graph ] && GFLAG="--graph"
mkdir -p $OUT
cd $R
timeout -k 10 200 python tools/train_bench.py --steps 5 --warmup 3 > $OUT/eager.json 2> $OUT/eager.err || exit $?
timeout -k 10 200 python tools/train_bench.py --steps 5 --warmup 3 --graph > $OUT/graph.json 2> $OUT/graph.err || exit $?
cat $OUT/eager.json $OUT/graph.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/tools/train_bench.py --steps 3 --warmup 4 $GFLAG > $OUT/kt.json 2> $OUT/kt.err || exit $?
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python tools/train_bench.py --steps 3 --warmup 4 $GFLAG (7 $MODE training steps, B=16, 256x256, 8 iters)" > $OUT/stats_$MODE.txt
python3 $R/tools/busy.py $DB --last-ms 150 > $OUT/busy_$MODE.txt 2>&1
rm -rf $OUT/kt
head -40 $OUT/stats_$MODE.txt; head -40 $OUT/busy_$MODE.txt
