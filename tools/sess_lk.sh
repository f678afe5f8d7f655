#!/bin/bash
# tile-region lookup: parity (lookup / decoder tests), lookup_bench A/B at configs[4] and [1],
# decoder bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lk; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
SCFLOW_LK_TILEREG=1 timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "lookup or pyramid or decoder or configs" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  SCFLOW_LK_TILEREG=$v timeout -k 10 120 python tools/lookup_bench.py --check > $OUT/lb4_$v.txt 2>&1 || exit $?
  SCFLOW_LK_TILEREG=$v timeout -k 10 120 python tools/lookup_bench.py --batch 16 --size 256 > $OUT/lb1_$v.txt 2>&1 || exit $?
  echo "tilereg=$v"; tail -2 $OUT/lb4_$v.txt; tail -2 $OUT/lb1_$v.txt
done
for v in 0 1 0 1; do
  SCFLOW_LK_TILEREG=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_$v.json 2>$OUT/bench_$v.err || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1]);print('tilereg=$v', d['value'], d['ms_per_step'], [(e['kernel'][:30], e.get('avg_launch_ms')) for e in d['rooflines_secondary'] if 'lookup' in e['kernel']])"
done
