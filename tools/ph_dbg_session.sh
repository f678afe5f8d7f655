#!/bin/bash
# fc2+heads kernel variants (SCFLOW_FC2H_DBG bits) under rocprofv3 → gpurun_out/ph_dbg/
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph_dbg
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for d in 0 1; do
  SCFLOW_FC2H_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/d$d -o run -- python3 $R/tools/ph_ab.py gnh > $OUT/d$d.log 2>&1 || exit $?
done
echo done
