"""Workgroup phase stamps of the pose head's two MFMA halo convs as the decoder launches them
(K split into partial slabs: conv1 224 → 128 /2 over ksplit 4, conv2 128 → 128 /2 with the
GroupNorm + ReLU applied on load over ksplit 8), B pairs at 32 × 32 features.

usage: python tools/enc_stamps.py [--batch 16] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scflow_amd import ops  # noqa: E402
from conv_bench import stamp_report  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    n, h = a.batch, 32
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, cin, hin, ks, norm in (("pose conv1 224->128 /2", 224, h, 4, False),
                                     ("pose conv2 128->128 /2 (GN on load)", 128, h // 2, 8, True)):
        w = (torch.randn(128, cin, 3, 3, generator=g) / (9 * cin) ** 0.5).to(dev)
        pk = ops.enc_conv_pack(w)
        x = torch.randn(n * hin * hin, cin, generator=g).to(dev)
        oh = hin // 2
        parts = torch.empty(ks * n * oh * oh, 128, device=dev)
        sc = torch.rand(n, cin, generator=g).to(dev) + 0.5 if norm else None
        sh = torch.randn(n, cin, generator=g).to(dev) * 0.1 if norm else None

        def run():
            ops.enc_conv(x, pk, None, n, hin, hin, cin, 128, 3, 2, 1, parts, in_scale=sc, in_shift=sh,
                         ksplit=ks)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        torch.cuda.synchronize()
        print(f"{name:40s} {s.elapsed_time(e) * 1e3 / a.reps:8.2f} us", flush=True)
        stamp_report(run)


if __name__ == "__main__":
    main()
