#!/bin/bash
# Lookup (and pyramid) counters at configs[4] (B=32, 512², 12 iters), tiled vs row-major pyramid:
# FETCH_SIZE and WRITE_SIZE passes (traffic per launch) and one SQ pass, each its own run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/lkc4; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer --batch 32 --size 512 --iters 12"
for v in ${VARIANTS:-tiled rowmajor}; do
  X=""; [ $v = rowmajor ] && X="--no-tiled-pyramid"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f_$v -o run -- python3 $R/bench.py $B $X > /dev/null 2> $OUT/f_$v.err || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$v -o run -- python3 $R/bench.py $B $X > /dev/null 2> $OUT/w_$v.err || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/s_$v -o run -- python3 $R/bench.py $B $X > /dev/null 2> $OUT/s_$v.err || exit 1
  python3 $R/tools/pmc_summary.py $(find $OUT/f_$v $OUT/w_$v $OUT/s_$v -name "*counter_collection.csv") | grep -iE "lookup|corr_gemm|avgpool" | cut -c1-700 > $OUT/summary_$v.txt
  python3 $R/tools/traffic_json.py $OUT/f_$v $OUT/w_$v --batch 32 --size 512 --iters 12 > $OUT/traffic_$v.json
  rm -rf $OUT/f_$v $OUT/w_$v $OUT/s_$v
done
cat $OUT/summary_*.txt
