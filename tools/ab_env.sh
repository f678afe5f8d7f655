# Same-box A/B of a training-step switch: GPU tests matching $K, then train_bench with $VAR=0 and
# default, twice each (alternating), and a kernel-trace of the default.
#   VAR=SCFLOW_TRAIN_GN_FUSED K="group_norm" bash tools/ab_env.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_train_ops.py tests/test_gpu_train.py} -k "$K" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
  tail -3 $O/t.log
fi
for i in 1 2; do
  env $VAR=0 timeout -k 10 200 python tools/train_bench.py --steps 8 --warmup 3 > $O/off$i.json 2>$O/off.err || exit $?
  timeout -k 10 200 python tools/train_bench.py --steps 8 --warmup 3 > $O/on$i.json 2>$O/on.err || exit $?
done
for f in $O/off1.json $O/off2.json $O/on1.json $O/on2.json; do echo "$f $(cat $f)"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/train_bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/$O/kt.json 2> $GRAFT_REPO_ROOT/$O/kt.err
