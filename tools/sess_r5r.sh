#!/bin/bash
# Round 5, session R: FETCH_SIZE / WRITE_SIZE passes at configs[1] and configs[4] again (the
# traffic JSONs of session P missed the GRU groups: kernel names carry "(anonymous namespace)::")
# + the full-resolution workgroup count A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_r5r; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer"
C4="--batch 32 --size 512 --iters 12"
pmc() {
  local t=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$t -o run -- python3 $R/bench.py "$@" > /dev/null 2> $OUT/$t.err || return 3
}
pmc fetch_c1 FETCH_SIZE $P || exit 3
pmc write_c1 WRITE_SIZE $P || exit 3
python3 $R/tools/traffic_json.py $OUT/fetch_c1 $OUT/write_c1 --batch 16 --size 256 --iters 8 > $OUT/traffic_b16_s256.json
pmc fetch_c4 FETCH_SIZE $P $C4 || exit 4
pmc write_c4 WRITE_SIZE $P $C4 || exit 4
python3 $R/tools/traffic_json.py $OUT/fetch_c4 $OUT/write_c4 --batch 32 --size 512 --iters 12 > $OUT/traffic_b32_s512.json
rm -rf $OUT/fetch_* $OUT/write_*
cd $R
bash tools/sess_r5q.sh || exit 5
