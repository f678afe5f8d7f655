#!/bin/bash
# STREAM ceiling + FETCH_SIZE / WRITE_SIZE calibration of the access patterns (tools/micro/stream.hip)
# usage (GPU box): bash tools/micro/stream_session.sh TAG  → gpurun_out/stream_TAG/
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stream_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/micro/stream > $OUT/stream.txt 2>&1 || exit $?
timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
cat $OUT/stream.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $R/tools/micro/stream 1 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $R/tools/micro/stream 1 > $OUT/write.log 2>&1 || exit $?
for c in fetch write; do
  f=$(find $OUT/$c -name "*counter_collection.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('$c', r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'])
" | tee -a $OUT/counters.txt
done
