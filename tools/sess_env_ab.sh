#!/bin/bash
# Decoder bench A/B of environment settings on one box, alternating, ROUNDS rounds:
# usage: tools/sess_env_ab.sh "A settings" "B settings" ["C settings" ...]   (e.g. "SCFLOW_WINO_SWZ=0")
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/env_ab; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for sets in "$@"; do
    i=$((i+1))
    env $sets timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$i.json 2>$OUT/b_$i.err || exit $?
    python3 -c "import json;d=json.loads(open('$OUT/b_$i.json').read().strip().splitlines()[-1]);print('[$sets]', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
