#!/bin/bash
# Profiles for the bench's decoder leg: kernel-trace stats + FETCH/WRITE PMC passes (separate
# runs) → gpurun_out/prof_TAG/{stats.txt,traffic.json}.  usage: tools/prof_session.sh TAG
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py $B > $OUT/bench_kt.json 2> $OUT/kt.err || exit $?
python3 $R/tools/stats_file.py $(find $OUT/kt -name "*.db" | head -1) "python bench.py $B" > $OUT/stats.txt
python3 $R/tools/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) 24 > $OUT/per_forward.txt  # 3 warmup + 10 timed + 1 + 10 secondary-timer forwards
python3 $R/tools/timeline.py $(find $OUT/kt -name "*.db" | head -1) --iteration 60 > $OUT/timeline.txt 2>&1
rm -rf $OUT/kt
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/fetch.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/write.err || exit $?
python3 $R/tools/traffic_json.py $OUT/fetch $OUT/write "wino5_kernel<0, 32, 2, 1>" "wino5_kernel<1, 32, 2, 1>" > $OUT/traffic.json
cat $OUT/traffic.json | head -5; head -12 $OUT/per_forward.txt
