set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/lkb; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train_ops.py -k "lookup" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
for i in 1 2; do
SCFLOW_LOOKUP_BWD_WIN=0 timeout -k 10 200 python tools/train_bench.py --steps 8 --warmup 3 > $O/off$i.json 2>$O/off.err || exit $?
timeout -k 10 200 python tools/train_bench.py --steps 8 --warmup 3 > $O/on$i.json 2>$O/on.err || exit $?
done
cat $O/*.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/train_bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$O/kt.json 2> $GRAFT_REPO_ROOT/$O/kt.err || exit $?
find $GRAFT_REPO_ROOT/$O/kt -name "*stats*.csv" | head -3 | xargs -I{} sh -c 'grep -i "lookup" {} || true'
