for cfg in "X=0" "SCFLOW_CONV_TILE_M=64" "SCFLOW_CONV_BK=8" "SCFLOW_CONV_TILE_M=64 SCFLOW_CONV_BK=8" "SCFLOW_CONV_TILE_M=128 SCFLOW_CONV_BK=8"; do
  env $cfg timeout -k 10 100 python tools/conv_bench.py --batch 16 > gpurun_out/c0.txt 2>&1 || exit 1
  echo "$cfg: $(grep 'corr_net.0' gpurun_out/c0.txt)"
done
