#!/bin/bash
# Progress-keyed wave priority in the Winograd kernels (F(4,5), F(2x2,3x3), F(4x4,3x3) GEMM) (WINO_PRIO=1, main library) vs without
# (lib/ab/noprio.so): parity, the GRU shapes alone, decoder at configs[1] / configs[4], alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r5au}; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
V=$R/scflow_amd/lib/ab/noprio.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "gru or wino or decoder or config" > $OUT/test.txt 2>&1
rc=$?; tail -2 $OUT/test.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in prio noprio; do
    L=""; [ $v = noprio ] && L=$V
    SCFLOW_LIB=$L timeout -k 10 200 python tools/conv_bench.py --only "+map,out_net,corr_net,heads,flow_net" --no-extras --reps 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$v$r.json 2>$OUT/b_$v$r.err || exit 3
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 6 --warmup 2 --batch 32 --size 512 --iters 12 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/c_$v$r.json 2>$OUT/c_$v$r.err || exit 4
    python3 -c "
import json
for f in ('b','c'):
    d=json.loads(open('$OUT/'+f+'_$v$r.json').read().strip().splitlines()[-1])
    print('$v', f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('launch_ms'))"
  done
done
