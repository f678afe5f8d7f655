#!/bin/bash
# Two PMC passes over tools/conv_bench.py (counters only); csv under gpurun_out/pmc_TAG/.
#   BENCH=tools/wgrad_bench.py GREP=wgrad tools/pmc_conv.sh w1   → the weight-gradient kernels
TAG=${1:-c1}
BENCH=${BENCH:-tools/conv_bench.py}
GREP=${GREP:-wino}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d $OUT/$name -o run -- "$@" \
      > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -- python3 $R/$BENCH --reps 3 || exit 1
run p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -- python3 $R/$BENCH --reps 3 || exit 1
python3 $R/tools/pmc_summary.py $(find $OUT/p1 $OUT/p2 -name "*counter_collection.csv") > $OUT/summary.txt 2>&1
grep -i "$GREP\|==" $OUT/summary.txt | cut -c1-900
