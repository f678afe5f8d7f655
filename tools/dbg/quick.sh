timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 -p no:cacheprovider > gpurun_out/quick_pytest.log 2>&1; tail -1 gpurun_out/quick_pytest.log
B="--steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" || exit 1
timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/cb_quick.txt && grep "thin\|flow_pred\|mask_pred\|smallcin\|7x7\|corr_net.0\|lookup\|sum" gpurun_out/cb_quick.txt
