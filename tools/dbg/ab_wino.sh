B="--steps 20 --warmup 3 --no-cpu-baseline --e2e-batch 0 --train-batch 0"
for v in 0 1 2; do
  if [ $v = 0 ]; then E=""; else E="SCFLOW_WINO_NBW=$v"; fi
  env $E timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" || exit 1
done
SCFLOW_CONV_WINO=5 timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wino5 only', d['value'], d['ms_per_step'])"
SCFLOW_CONV_WINO=3 timeout -k 10 120 python bench.py $B | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wino3 only', d['value'], d['ms_per_step'])"
