#!/bin/bash
# Round 5, session AO: bias prefetch in the fused lookup + corr_net.0 and the wide 1×1 conv: the whole GPU
# suite, then the decoder A/B against the previous box-to-box range and a kernel trace.
set -o pipefail
O=gpurun_out/r5ao; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/ab_bench.py --rounds 7 --steps 10 > $O/ab.txt 2>&1 || exit 3
cd /tmp && R=${GRAFT_REPO_ROOT}; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $R/$O/bench_kt.json 2> $R/$O/kt.err || exit 5
DB=$(find $R/$O/kt -name "*.db" | head -1); python3 $R/tools/timeline.py $DB --iteration 60 > $R/$O/timeline_c1.txt 2>&1; python3 $R/tools/prof_summary.py $DB 24 > $R/$O/per_forward_c1.txt; rm -rf $R/$O/kt
