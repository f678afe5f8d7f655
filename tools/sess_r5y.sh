#!/bin/bash
# Round 5, session Y: small-cin MFMA conv phases (workgroup stamps) + in-decoder trace.
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "flow_net.0,mask_enc.0" > $O/conv.txt 2>&1 || exit 3
SCFLOW_SMALLCIN_SPLIT=1 timeout -k 10 120 python -u tools/conv_bench.py --no-extras --stamps --only "flow_net.0" > $O/conv_split.txt 2>&1 || exit 3
