#!/bin/bash
# training-step attribution at HEAD: torch.profiler glue sites (by Python stack) and the
# rocprofv3 kernel-trace summary of 5 eager training steps
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/train_$1
mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python tools/train_torchprof.py --stack 4 --rows 60 > $OUT/glue.txt 2>&1 || exit $?
head -80 $OUT/glue.txt
bash tools/gpu_session.sh $1 trainprof || exit $?
cp $R/gpurun_out/train_stats_$1.txt $OUT/ 2>/dev/null; head -30 $OUT/train_stats_$1.txt
