set -o pipefail
export TMPDIR=/tmp
SCFLOW_TRAIN_ERRS=gpurun_out/train_errs_c3.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_r03a.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err
echo "bench rc=$?"; head -c 1500 gpurun_out/bench_r03a.json
