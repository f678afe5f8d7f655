"""Time scflow_conv_wgrad against HIP im2col + hipBLASLt matmul on the training step's shapes.

usage: python tools/wgrad_bench.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (n, h, w, cin0, cin1, cout, kh, kw, stride, pad) at B=16 pairs
SHAPES = [
    (48, 128, 128, 64, 0, 64, 3, 3, 1, (1, 1)),    # encoder layer1 (32 feature + 16 context images)
    (16, 32, 32, 128, 0, 256, 3, 3, 1, (1, 1)),    # flow/mask head 3x3 128->256
    (16, 32, 32, 128, 128, 256, 1, 5, 1, (0, 2)),  # GRU zr 1x5 (h ⊕ motion)
    (16, 32, 32, 128, 128, 256, 5, 1, 1, (2, 0)),  # GRU zr 5x1
    (16, 32, 32, 256, 0, 192, 3, 3, 1, (1, 1)),    # corr_net.1
    (16, 32, 32, 324, 0, 256, 1, 1, 1, (0, 0)),    # corr_net.0
    (48, 64, 64, 96, 0, 96, 3, 3, 1, (1, 1)),      # encoder layer2
    (16, 32, 32, 224, 0, 128, 3, 3, 2, (1, 1)),    # pose head conv1 (stride 2)
    (48, 128, 128, 64, 0, 96, 3, 3, 2, (1, 1)),    # encoder layer2.0 conv1 (stride 2)
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from scflow_amd import ops
    dev = torch.device("cuda", 0)
    tot_k = tot_g = 0.0
    for (n, h, w, c0, c1, cout, kh, kw, s, (ph, pw)) in SHAPES:
        oh, ow = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
        x0 = torch.randn(n, h, w, c0, device=dev)
        x1 = torch.randn(n, h, w, c1, device=dev) if c1 else None
        dy = torch.randn(n * oh * ow, cout, device=dev)
        dw = torch.empty(cout, c0 + c1, kh, kw, device=dev)
        db = torch.empty(cout, device=dev)
        flops = 2.0 * n * oh * ow * cout * (c0 + c1) * kh * kw

        def k():
            ops.conv_wgrad(dy, x0, x1, dw, db, n, h, w, kh, kw, s, ph, pw)

        def g():
            x = x0 if x1 is None else torch.cat([x0, x1], -1)
            cols = ops.im2col(x, n, h, w, c0 + c1, kh, kw, s, ph, pw)
            torch.matmul(dy.t(), cols)
            dy.sum(0)

        res = []
        for fn in (k, g):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / a.reps)
        tot_k += res[0]
        tot_g += res[1]
        print(f"{str((n, h, w, c0, c1, cout, kh, kw, s)):44s} {flops / 1e9:7.2f} GF  wgrad {res[0]:7.3f} ms "
              f"({flops / res[0] / 1e9:6.1f} TF/s)  im2col+mm {res[1]:7.3f} ms ({flops / res[1] / 1e9:6.1f} TF/s)")
    print(f"total wgrad {tot_k:.3f} ms  im2col+mm {tot_g:.3f} ms")


if __name__ == "__main__":
    main()
