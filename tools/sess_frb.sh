#!/bin/bash
# workgroups per image of the deferred full-resolution launch: decoder bench per setting, 2 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/frb; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
for r in 1 2; do for b in 64 16 32 8 128; do
  SCFLOW_FULLRES_BLOCKS=$b timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$b.json 2>$OUT/b_$b.err || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/b_$b.json').read().strip().splitlines()[-1]);print('blocks=$b', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
done; done
