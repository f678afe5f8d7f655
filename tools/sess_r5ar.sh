#!/bin/bash
# Training-step per-step times in order, three bench legs (is the slow step systematic?).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ar; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --e2e-batch 0 > $OUT/b$i.json 2> $OUT/b$i.err || exit $i
  python3 -c "import json;d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]);print(d['training_step']['per_step_ms'])"
done
