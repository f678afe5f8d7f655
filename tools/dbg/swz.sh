R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/swz; mkdir -p $O
SCFLOW_WINO_SWZ=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or gru" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in 0 1 2 4 8; do
  SCFLOW_WINO_SWZ=$c timeout -k 10 200 python tools/conv_bench.py --batch 16 > $O/cb_$c.txt 2>&1 || exit 2
done
