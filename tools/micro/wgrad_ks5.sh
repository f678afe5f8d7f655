# 1×5 / 5×1 weight gradients with one vs two wave sets (SCFLOW_WGRAD_KS5): parity tests, then timing
set -o pipefail
SCFLOW_WGRAD_KS5=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train_ops.py -k "wgrad or conv_backward" > gpurun_out/ks5_t.log 2>&1 || { tail -20 gpurun_out/ks5_t.log; exit 1; }
tail -2 gpurun_out/ks5_t.log
for v in 0 1 2 0 1 2; do echo "KS5=$v"; SCFLOW_WGRAD_KS5=$v timeout -k 10 60 python tools/micro/wgrad_bench.py 2>&1 | grep -E "  256  (256|128)  (1  5|5  1) 1" || exit 1; done
