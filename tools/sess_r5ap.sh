#!/bin/bash
# A/B: the pose head's conv1 split into a main-stream launch (h + Δflow features) and a
# side-stream slab (mask features) before the join, vs one launch after it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ap; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "decoder or pose or config or refine or e2e" > $OUT/test.txt 2>&1
rc=$?; tail -2 $OUT/test.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py --rounds 7 split_trunk_side=1,0 > $OUT/ab.txt 2>&1 || exit 3
cat $OUT/ab.txt
timeout -k 10 300 python tools/ab_bench.py --rounds 5 --batch 32 --size 512 --iters 12 split_trunk_side=1,0 > $OUT/ab_c4.txt 2>&1 || exit 4
cat $OUT/ab_c4.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_kt.json 2> $OUT/kt.err || exit 5
DB=$(find $OUT/kt -name "*.db" | head -1)
python3 $R/tools/timeline.py $DB --iteration 60 > $OUT/timeline_c1.txt 2>&1
rm -rf $OUT/kt
tail -14 $OUT/timeline_c1.txt
