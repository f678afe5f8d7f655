# Training-step A/B on one box: alternating runs of tools/train_bench.py under env settings
# A and B (e.g. A="SCFLOW_DEFER_LINEAR=1" B="SCFLOW_DEFER_LINEAR=0"), ROUNDS pairs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/train_ab
mkdir -p $OUT
cd $R
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    eval "sets=\$$v"
    r=$(env $sets timeout -k 10 200 python tools/train_bench.py --steps 5 --warmup 3 2>/dev/null | tail -1) || exit $?
    echo "$v [$sets] $r" | tee -a $OUT/ab.txt
  done
done
