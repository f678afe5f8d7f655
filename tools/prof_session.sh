#!/bin/bash
# Profiles for the bench's decoder leg: kernel-trace stats + FETCH/WRITE PMC passes (separate
# runs) at configs[1] (B=16, 256², 8 iters) and configs[4] (B=32, 512², 12 iters)
#   → gpurun_out/prof_TAG/{stats.txt,per_forward.txt,timeline.txt,traffic_b16_s256.json,traffic_b32_s512.json}
# usage: tools/prof_session.sh TAG
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py $B > $OUT/bench_kt.json 2> $OUT/kt.err || exit $?
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python bench.py $B" > $OUT/stats.txt
python3 $R/tools/prof_summary.py $DB 24 > $OUT/per_forward.txt  # 3 warmup + 10 timed + 1 + 10 secondary-timer forwards
python3 $R/tools/timeline.py $DB --iteration 60 > $OUT/timeline.txt 2>&1
rm -rf $OUT/kt
pmc() {  # tag, bench args
  local t=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$t -o run -- python3 $R/bench.py "$@" > /dev/null 2> $OUT/fetch_$t.err || return $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$t -o run -- python3 $R/bench.py "$@" > /dev/null 2> $OUT/write_$t.err || return $?
}
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer"
pmc c1 $P || exit $?
python3 $R/tools/traffic_json.py $OUT/fetch_c1 $OUT/write_c1 --batch 16 --size 256 --iters 8 > $OUT/traffic_b16_s256.json
pmc c4 $P --size 512 --batch 32 --iters 12 || exit $?
python3 $R/tools/traffic_json.py $OUT/fetch_c4 $OUT/write_c4 --batch 32 --size 512 --iters 12 > $OUT/traffic_b32_s512.json
rm -rf $OUT/fetch_* $OUT/write_*
head -c 600 $OUT/traffic_b16_s256.json; head -12 $OUT/per_forward.txt
