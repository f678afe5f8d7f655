#!/bin/bash
# Round 5, session E: the whole GPU suite (after the opt-in removals; F(4x4) tests), then the
# F(4x4,3x3) stamps / transform split / decoder A/B.
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfs --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
bash tools/sess_w4c.sh r5e_w4
