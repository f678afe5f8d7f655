"""Standalone timing of the correlation branch's first two operators at the decoder's shapes:
the tiled lookup, corr_net.0 on the direct 1×1 kernel (bk 16) and on the wide 1×1 kernel
(SCFLOW_CONV_1X1W), and the two fused (scflow_corr_lookup_conv1x1).

    python tools/lookup_conv_bench.py [--batch 16 --size 32] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=32, help="feature map side")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from scflow_amd import _lib, ops
    from scflow_amd.modules import ConvRunner
    n, h, w = a.batch, a.size, a.size
    M = n * h * w
    g = torch.Generator().manual_seed(0)
    f1 = torch.randn(n, 256, h, w, generator=g).cuda()
    f2 = torch.randn(n, 256, h, w, generator=g).cuda()
    pyr = ops.corr_pyramid_tiled(f1, f2, 4)
    flow = ((torch.rand(M, 2, generator=g) - 0.5) * 8).cuda()
    conv = torch.nn.Conv2d(324, 256, 1).cuda()
    r = ConvRunner([conv], "ReLU")
    corr = torch.empty(M, 324, device="cuda")
    out = torch.empty(M, 256, device="cuda")
    pk16, bias = r.packed(324, 0, w, 16)
    pkw, _ = r.packed(324, 0, w, _lib.CONV_1X1W)
    pk16 = pk16.clone()

    cases = {
        "lookup (tiled)": lambda: ops.corr_lookup(pyr, flow, n, h, w, 4, 4, out=ops.Chan.whole(corr),
                                                  flow_layout="nhwc", tiled=True),
        "corr_net.0 conv1x1_kernel": lambda: ops.conv2d(ops.Chan.whole(corr), pk16, bias, n, h, w, 256, 1,
                                                         1, 0, 0, "ReLU", out=ops.Chan.whole(out), bk=16),
        "corr_net.0 conv1x1w_kernel": lambda: ops.conv2d(ops.Chan.whole(corr), pkw, bias, n, h, w, 256, 1,
                                                          1, 0, 0, "ReLU", out=ops.Chan.whole(out),
                                                          bk=_lib.CONV_1X1W),
        "fused lookup+corr_net.0": lambda: ops.corr_lookup_conv1x1(pyr, flow, pkw, bias, ops.Chan.whole(out),
                                                                   n, h, w, 4, 4, 256),
    }
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = 2.0 * M * 324 * 256
        print(f"B={n} {h}x{w} {name:28s} {us:8.1f} us   {fl / us / 1e6:6.1f} TF(GEMM-equiv)", flush=True)


if __name__ == "__main__":
    main()
