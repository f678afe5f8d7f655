#!/bin/bash
# HEAD evidence for the default decoder path (§8(d)): kernel trace + stats and per-iteration
# timeline at configs[1]; kernel stats at configs[4]; FETCH_SIZE / WRITE_SIZE passes at both
# (→ traffic JSONs); an SQ pass (MFMA busy, LDS bank conflicts, waits) over the decoder at both.
# Each rocprofv3 pass is its own run.  usage: tools/prof_r5.sh TAG  → gpurun_out/prof_TAG/
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
C4="--batch 32 --size 512 --iters 12"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py $B > $OUT/bench_kt_c1.json 2> $OUT/kt.err || exit 1
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python bench.py $B" > $OUT/stats_c1.txt
python3 $R/tools/prof_summary.py $DB 24 > $OUT/per_forward_c1.txt
python3 $R/tools/timeline.py $DB --iteration 60 > $OUT/timeline_c1.txt 2>&1
rm -rf $OUT/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt4 -o run -- python3 $R/bench.py $B $C4 > $OUT/bench_kt_c4.json 2> $OUT/kt4.err || exit 2
DB=$(find $OUT/kt4 -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python bench.py $B $C4" > $OUT/stats_c4.txt
python3 $R/tools/prof_summary.py $DB 24 > $OUT/per_forward_c4.txt
rm -rf $OUT/kt4
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer"
pmc() {  # tag, counters (one pass), bench args
  local t=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$t -o run -- python3 $R/bench.py "$@" > /dev/null 2> $OUT/$t.err || return 3
}
pmc fetch_c1 FETCH_SIZE $P || exit 3
pmc write_c1 WRITE_SIZE $P || exit 3
python3 $R/tools/traffic_json.py $OUT/fetch_c1 $OUT/write_c1 --batch 16 --size 256 --iters 8 > $OUT/traffic_b16_s256.json
pmc fetch_c4 FETCH_SIZE $P $C4 || exit 4
pmc write_c4 WRITE_SIZE $P $C4 || exit 4
python3 $R/tools/traffic_json.py $OUT/fetch_c4 $OUT/write_c4 --batch 32 --size 512 --iters 12 > $OUT/traffic_b32_s512.json
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
pmc sq_c1 "$SQ" $P || exit 5
pmc sq_c4 "$SQ" $P $C4 || exit 6
for t in c1 c4; do
  python3 $R/tools/pmc_summary.py $(find $OUT/fetch_$t $OUT/write_$t $OUT/sq_$t -name "*counter_collection.csv") > $OUT/pmc_$t.txt
done
rm -rf $OUT/fetch_* $OUT/write_* $OUT/sq_*
head -c 400 $OUT/traffic_b16_s256.json; head -12 $OUT/per_forward_c1.txt
