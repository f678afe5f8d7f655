#!/bin/bash
# Progress-keyed wave priority in enc_conv_kernel (ENC_PRIO=1, main library) vs without
# (lib/ab/encnoprio.so): parity, pose head alone, decoder configs[1] / configs[4], end to end.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5aw; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
V=$R/scflow_amd/lib/ab/encnoprio.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "pose or encoder or config or refine or e2e" > $OUT/test.txt 2>&1
rc=$?; tail -2 $OUT/test.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in prio noprio; do
    L=""; [ $v = noprio ] && L=$V
    SCFLOW_LIB=$L timeout -k 10 200 python tools/ph_bench.py 2>&1 | grep "enc_conv\|whole" | sed "s/^/$v /"
    SCFLOW_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --train-batch 0 > $OUT/b_$v$r.json 2>$OUT/b_$v$r.err || exit 3
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 6 --warmup 2 --batch 32 --size 512 --iters 12 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/c_$v$r.json 2>$OUT/c_$v$r.err || exit 4
    python3 -c "
import json
for f in ('b','c'):
    d=json.loads(open('$OUT/'+f+'_$v$r.json').read().strip().splitlines()[-1])
    e=d.get('end_to_end',{})
    print('$v', f, d['value'], d['ms_per_step'], e.get('value'), e.get('ms_per_step'))"
  done
done
