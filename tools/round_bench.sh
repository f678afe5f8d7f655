set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python bench.py > gpurun_out/bench_r02e.json 2> gpurun_out/bench_r02e.err || exit $?
cat gpurun_out/bench_r02e.json | head -c 400; echo
bash tools/prof_session.sh r02e || exit $?
