"""Pose-head (a7) trunk variants in isolation, for rocprofv3 kernel stats.

usage: python tools/ph_ab.py VARIANT [--batch 16] [--reps 200]
  VARIANT: old  (GroupNorm launches, FC2 and heads separate)
           gn   (fused-statistics trunk, FC2 and heads separate)
           gnh  (fused-statistics trunk, FC2 + heads in one launch)
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scflow_amd import MODELS, synthetic  # noqa: E402
from scflow_amd.ops import Chan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant", choices=["old", "gn", "gnh"])
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    n, h, w = a.batch, 32, 32
    head = MODELS.build(dict(type="MultiClassPoseHead", num_class=21, in_channels=224, net_type="Basic",
                             rotation_mode="ortho6d", norm_cfg=dict(type="GN", num_groups=32),
                             act_cfg=dict(type="ReLU")))
    synthetic.fill_module_(head, seed=3)
    head = head.cuda().eval()
    head.fused_gn = a.variant != "old"
    head.fused_fc2_heads = a.variant == "gnh"
    hx = torch.randn(n * h * w, 384, device="cuda")
    fm = torch.randn(n * h * w, 96, device="cuda")
    label = torch.randint(0, 21, (n,), device="cuda")
    ws = []
    x = head.trunk_hip(Chan(hx, 0, 128), Chan.whole(fm), n, h, w, ws=ws)
    drot = torch.empty(n, 6, device="cuda")
    dt = torch.empty(n, 3, device="cuda")
    for _ in range(5):
        head.trunk_hip(Chan(hx, 0, 128), Chan.whole(fm), n, h, w, ws=ws)
        head.heads_hip(x, label, drot, dt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        x = head.trunk_hip(Chan(hx, 0, 128), Chan.whole(fm), n, h, w)
        head.heads_hip(x, label, drot, dt)
    torch.cuda.synchronize()
    print(f"{a.variant}: {(time.perf_counter() - t0) / a.reps * 1e6:.1f} us per trunk+heads (host-inclusive)")


if __name__ == "__main__":
    main()
