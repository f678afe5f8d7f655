#!/bin/bash
# A/B of a library variant against the default build on one GPU box: parity of the variant, then
# a conv_bench shape and the decoder bench, alternating, two rounds.
# Build the variant here first (not on the box):  tools/build_variant.sh NAME FILE.hip "-DFLAG=1"
# usage: tools/sess_variant.sh NAME "PYTEST -k EXPR" "CONV_BENCH --only EXPR"
NAME=$1; K=${2:-"conv2d or decoder"}; ONLY=${3:-"flow_pred"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/variant_$NAME; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
V=$R/scflow_amd/lib/ab/$NAME.so
[ -f $V ] || { echo "missing $V"; exit 2; }
SCFLOW_LIB=$V timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base $NAME; do
    L=""; [ $v != base ] && L=$V
    SCFLOW_LIB=$L timeout -k 10 200 python tools/conv_bench.py --only "$ONLY" --no-extras --reps 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
    SCFLOW_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/b_$v.json 2>$OUT/b_$v.err || exit $?
    python3 -c "import json;d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])"
  done
done
