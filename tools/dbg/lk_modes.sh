for m in 0 4 8; do LK_DBG=$m timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/lkm_$m.txt 2>&1 || exit 1; echo "mode $m $(grep 'corr lookup' gpurun_out/lkm_$m.txt)"; done
