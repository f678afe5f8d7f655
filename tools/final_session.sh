#!/bin/bash
# End-of-round GPU session: parity tests, bench (all legs), profiles, configs[4] bench line.
# usage: tools/final_session.sh TAG
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_session.sh $TAG test || exit $?
bash $R/tools/gpu_session.sh $TAG bench || exit $?
bash $R/tools/prof_session.sh $TAG || exit $?
timeout -k 10 400 python $R/bench.py --size 512 --batch 32 --iters 12 --steps 5 --warmup 2 \
    --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $R/gpurun_out/bench_cfg5_$TAG.json \
    2> $R/gpurun_out/bench_cfg5_$TAG.err || exit $?
head -c 400 $R/gpurun_out/bench_cfg5_$TAG.json
