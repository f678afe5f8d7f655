#!/bin/bash
# A/B of the MFMA stem's output rows per workgroup (SCFLOW_STEM_ROWS): encoder parity at each
# setting, then a kernel-trace profile of the end-to-end leg → gpurun_out/stem_rows.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/stem_rows.txt
for rows in ${STEM_ROWS_LIST:-4 8 16}; do
  SCFLOW_STEM_ROWS=$rows timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu $R/tests/test_gpu_encoder.py > $OUT/stem_rows_$rows.log 2>&1 || { tail -20 $OUT/stem_rows_$rows.log; exit 1; }
  echo "rows=$rows $(tail -1 $OUT/stem_rows_$rows.log)" >> $OUT/stem_rows.txt
  cd /tmp
  SCFLOW_STEM_ROWS=$rows timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sr$rows -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 3 --train-batch 0 > $OUT/sr$rows.json 2> $OUT/sr$rows.err || exit $?
  DB=$(find $OUT/sr$rows -name "*.db" | head -1)
  python3 $R/tools/stats_file.py $DB "rows=$rows" | grep -E "stem" >> $OUT/stem_rows.txt
  rm -rf $OUT/sr$rows
  cd $R
done
cat $OUT/stem_rows.txt
