#!/bin/bash
# Round 5, session AK: phases of the pose head's MFMA halo convs (workgroup stamps).
set -o pipefail
O=gpurun_out/r5ak; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/enc_stamps.py > $O/stamps.txt 2>&1 || exit 3
