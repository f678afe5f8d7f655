timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 -p no:cacheprovider > gpurun_out/quick_pytest.log 2>&1; tail -1 gpurun_out/quick_pytest.log
grep -q " passed" gpurun_out/quick_pytest.log && ! grep -q "failed\|error" gpurun_out/quick_pytest.log || exit 1
timeout -k 10 300 python tools/ab_bench.py --rounds 7 device_scope_events=1,0 > gpurun_out/ab_ev.txt 2>&1 || exit 1
tail -2 gpurun_out/ab_ev.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ev -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > /dev/null 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/timeline.py $GRAFT_REPO_ROOT/gpurun_out/ev/run_results.db --iteration 30
