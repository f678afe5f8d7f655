#!/bin/bash
# thin-conv variants: isolated timings (conv_bench) of the small decoder convs, then the decoder
# bench with the base library and the THINF_UNROLL=4 variant (tools/build_variant.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/thin; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
SCFLOW_LIB=$R/scflow_amd/lib/ab/thinxcd.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv2d or decoder" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc


for r in 1 2; do
  for v in base thinxcd; do
    L=""; [ $v != base ] && L=$R/scflow_amd/lib/ab/$v.so
    SCFLOW_LIB=$L timeout -k 10 200 python tools/conv_bench.py --only "flow_pred" --no-extras --reps 50 2>&1 | grep flow_pred | sed "s/^/$v /"
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$v.json 2>$OUT/b_$v.err || exit $?
    python3 -c "import json;d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])"
  done
done
