# lookup rewrite: GPU parity tests, bench, kernel-trace summary
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 -p no:cacheprovider > gpurun_out/quick_pytest.log 2>&1; tail -3 gpurun_out/quick_pytest.log
grep -q " passed" gpurun_out/quick_pytest.log && ! grep -q "failed\|error" gpurun_out/quick_pytest.log || exit 1
B="--steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lk -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > /dev/null 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/lk/run_results.db 7 | head -14
python3 $GRAFT_REPO_ROOT/tools/timeline.py $GRAFT_REPO_ROOT/gpurun_out/lk/run_results.db --iteration 30 | tail -1
