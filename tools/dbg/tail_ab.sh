timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 -p no:cacheprovider > gpurun_out/quick_pytest.log 2>&1; tail -1 gpurun_out/quick_pytest.log
grep -q " passed" gpurun_out/quick_pytest.log && ! grep -q "failed\|error" gpurun_out/quick_pytest.log || exit 1
timeout -k 10 300 python tools/ab_bench.py --rounds 7 fuse_tail=1,0 > gpurun_out/ab_tail.txt 2>&1 || exit 1
tail -2 gpurun_out/ab_tail.txt
