#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only + kernel names), csv output.
# usage: tools/pmc_session.sh TAG  → gpurun_out/pmc_TAG/{conv_p1,conv_p2,bench_fetch,bench_write}
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters..., -- cmd
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -k 10 300 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d $OUT/$name -o run -- "$@" \
      > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run conv_p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -- python3 $R/tools/conv_bench.py --reps 3 || exit 1
run conv_p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -- python3 $R/tools/conv_bench.py --reps 3 || exit 1
run bench_fetch FETCH_SIZE -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 || exit 1
run bench_write WRITE_SIZE -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 || exit 1
