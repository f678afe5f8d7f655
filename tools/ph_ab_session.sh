#!/bin/bash
# kernel stats of the pose-head variants (tools/ph_ab.py) → gpurun_out/ph_ab/
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in old gn gnh; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run -- python3 $R/tools/ph_ab.py $v > $OUT/$v.log 2>&1 || exit $?
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; cat $OUT/$v.log | tail -1
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows:
    print('%9.2f us  %6s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:70]))
" | tee $OUT/$v.txt
done
