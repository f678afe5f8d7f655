#!/bin/bash
# Host lead per kernel (rocprofv3 --kernel-trace --hip-trace, no counters) at configs[1].
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5aq; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $OUT/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer > $OUT/bench.json 2> $OUT/kt.err || exit 1
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/host_lead.py $DB --iteration 60 > $OUT/lead_c1.txt 2>&1
python3 $R/tools/timeline.py $DB --iteration 60 > $OUT/timeline_c1.txt 2>&1
rm -rf $OUT/kt
cat $OUT/lead_c1.txt
