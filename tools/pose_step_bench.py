"""The iteration tail's pose step alone (scflow_pose_step / _part) at a BASELINE config, HIP-event
timed over recorded launches: parts 1 (full resolution: pose flow, ×8 flow and mask), 2 (the next
iteration's ↓8 flow) and 3 (both), against the full-resolution part's algorithmic bytes.

usage: python tools/pose_step_bench.py [--batch 16] [--size 256] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    dev = torch.device("cuda", 0)
    n, H = a.batch, a.size
    W, h, w = H, H // 8, H // 8
    g = torch.Generator(device="cpu").manual_seed(3)
    # 40 % of the pixels on the object (the rest invalid), depths 0.5–1.5
    depth = torch.where(torch.rand(n, H, W, generator=g) < 0.4, torch.rand(n, H, W, generator=g) + 0.5,
                        torch.zeros(n, H, W))
    depth = depth.to(dev).float().contiguous()
    K = torch.tensor([[572.4, 0, 128.0], [0, 573.6, 128.0], [0, 0, 1]]).repeat(n, 1, 1).to(dev)
    R = torch.eye(3).repeat(n, 1, 1).to(dev)
    t = torch.tensor([0.0, 0.0, 1.0]).repeat(n, 1).to(dev)
    pts = ops.lift_points(depth, K, R, t)
    drot = (torch.randn(n, 6, generator=g) * 0.01 + torch.tensor([1.0, 0, 0, 0, 1.0, 0])).to(dev)
    dt = (torch.randn(n, 3, generator=g) * 0.01).to(dev)
    lr = torch.randn(n, h, w, 2, generator=g).to(dev)
    delta = torch.randn(n, h, w, 2, generator=g).to(dev)
    mask = torch.rand(n, h, w, generator=g).to(dev)
    Ro, to = torch.empty(n, 3, 3, device=dev), torch.empty(n, 3, device=dev)
    flow = torch.empty(n, 2, H, W, device=dev)
    fup = torch.empty(n, 2, H, W, device=dev)
    mup = torch.empty(n, 1, H, W, device=dev)
    lr2 = torch.empty(n, h, w, 2, device=dev)
    step = (drot, dt, R, t, K, pts, Ro, to, flow, 400.0, lr, delta, mask, fup, mup, h, w, 8.0)
    nxt = dict(lr_next=Chan.whole(lr2.view(n * h * w, 2)))
    px = n * H * W
    full_bytes = px * (16 + 8 + 8 + 4)
    for parts in (1, 2, 3):
        calls = []
        with ops.binding(calls):
            ops.pose_step(*step, **nxt, parts=parts)
        for _ in range(5):
            for c in calls:
                c()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            for c in calls:
                c()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        extra = f", {full_bytes / us / 1e3:.0f} GB/s of the full-resolution part's {full_bytes / 1e6:.1f} MB" \
            if parts & 1 else ""
        print(f"pose_step parts={parts}: {us:.1f} us/launch{extra}")


if __name__ == "__main__":
    main()
