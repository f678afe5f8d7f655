timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/cb_auto.txt || exit 1
SCFLOW_WINO_NBW=1 timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/cb_n1.txt || exit 1
SCFLOW_WINO_NBW=2 timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/cb_n2.txt || exit 1
paste -d'|' gpurun_out/cb_n1.txt gpurun_out/cb_n2.txt | grep -v amdgpu | cut -c1-50,51-130
