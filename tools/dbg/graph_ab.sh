B="--steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" || exit 1
timeout -k 10 120 python bench.py $B --graph | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" || exit 1
