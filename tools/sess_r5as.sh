#!/bin/bash
# Tile-row lookup sampling remap (one pixel per 32-lane half, region row pitch 12): parity, the
# lookup alone and the decoder at configs[4] against the previous kernel (lib/ab/lkold.so),
# alternating, then the SQ PMC pass of the new one.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5as; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
OLD=$R/scflow_amd/lib/ab/lkold.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "lookup or config or corr" > $OUT/test.txt 2>&1
rc=$?; tail -2 $OUT/test.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in old new; do
    L=""; [ $v = old ] && L=$OLD
    SCFLOW_LIB=$L timeout -k 10 200 python tools/lookup_bench.py --batch 32 --size 512 --reps 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 3
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --batch 32 --size 512 --iters 12 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$v$r.json 2>$OUT/b_$v$r.err || exit 4
    python3 -c "
import json;d=json.loads(open('$OUT/b_$v$r.json').read().strip().splitlines()[-1])
lk=[e for e in d['rooflines_secondary'] if 'lookup' in e['kernel']]
print('$v', d['value'], d['ms_per_step'], [(e.get('avg_launch_ms'), e.get('frac')) for e in lk])"
  done
done
cd /tmp
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer --batch 32 --size 512 --iters 12"
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/sq.err || exit 5
python3 $R/tools/pmc_summary.py $(find $OUT/sq -name "*counter_collection.csv") | grep -i lookup > $OUT/pmc_lookup_c4.txt
rm -rf $OUT/sq
cat $OUT/pmc_lookup_c4.txt
