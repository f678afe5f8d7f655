"""Weight-gradient calls (functions._weight_grad: the wgrad kernels, or im2col + GEMM outside
their shape set) of the training step, timed alone (HIP events over 20 calls each):
the decoder / pose-head / encoder shapes of configs[3] (B=16, 32² decoder, 128² encoder).

    python tools/micro/wgrad_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # n, h, w, cin, cout, kh, kw, stride
    (16, 32, 32, 256, 2, 3, 3, 1), (16, 32, 32, 1, 64, 3, 3, 1), (16, 32, 32, 256, 1, 1, 1, 1),
    (16, 32, 32, 64, 32, 3, 3, 1), (16, 32, 32, 128, 64, 3, 3, 1), (16, 32, 32, 256, 128, 3, 3, 1),
    (16, 32, 32, 128, 256, 3, 3, 1), (16, 32, 32, 256, 192, 3, 3, 1), (16, 32, 32, 256, 256, 1, 5, 1),
    (16, 32, 32, 256, 128, 5, 1, 1),
    (16, 32, 32, 256, 256, 5, 1, 1), (16, 32, 32, 256, 128, 1, 5, 1), (16, 32, 32, 324, 256, 1, 1, 1), (16, 32, 32, 224, 128, 3, 3, 2),
    (16, 16, 16, 128, 128, 3, 3, 2), (16, 8, 8, 128, 128, 3, 3, 2), (32, 128, 128, 64, 64, 3, 3, 1),
    (32, 64, 64, 96, 96, 3, 3, 1), (16, 32, 32, 256, 128, 3, 3, 1), (16, 32, 32, 2, 128, 7, 7, 1),
    (32, 256, 256, 3, 64, 7, 7, 2),
]


def main():
    from scflow_amd.train.functions import _weight_grad
    g = torch.Generator().manual_seed(0)
    print(" n   h   w  cin cout kh kw s |   us/call   TF/s")
    for n, h, w, cin, cout, kh, kw, s in SHAPES:
        ph, pw = kh // 2, kw // 2
        oh, ow = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
        x = torch.randn(n, h, w, cin, generator=g).cuda()
        dy = torch.randn(n * oh * ow, cout, generator=g).cuda()
        wt = torch.empty(cout, cin, kh, kw, device="cuda")
        dy = dy.view(n, oh, ow, cout)
        try:
            for _ in range(3):
                _weight_grad(dy, x, None, wt, s, ph, pw, True)
        except Exception as e:  # noqa: BLE001 — shapes outside the kernel set
            print(f"{n:3d} {h:3d} {w:3d} {cin:4d} {cout:4d} {kh:2d} {kw:2d} {s} | unsupported ({e})")
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2_000_000)
        e0.record()
        for _ in range(20):
            _weight_grad(dy, x, None, wt, s, ph, pw, True)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        fl = 2.0 * n * oh * ow * cout * cin * kh * kw
        print(f"{n:3d} {h:3d} {w:3d} {cin:4d} {cout:4d} {kh:2d} {kw:2d} {s} | {us:9.1f} {fl / us / 1e6:6.1f}")


if __name__ == "__main__":
    main()
