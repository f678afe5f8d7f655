"""corr_net.0's 1×1 conv (324 → 256 at B=16, 32×32; and its 256 → 324 dX) on the conv dispatch
(conv_mfma) against the plain fp32 MFMA GEMM (scflow_gemm_f32), HIP-event timed.

usage: python tools/conv1x1_bench.py [--batch 16] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    dev = torch.device("cuda", 0)
    n, h, w = a.batch, 32, 32
    for cin, cout in ((324, 256), (256, 324), (128, 256), (256, 128)):
        x = torch.randn(n * h * w, cin, device=dev)
        wt = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        out = torch.empty(n * h * w, cout, device=dev)
        bk = ops.conv_pick_bk(n, h, w, cin, 0, cout, 1, 1, 0, 0, 1)
        packed = ops.pack_conv_weight(wt, cin, 0, w, 1, bk)
        us_c = timeit(lambda: ops.conv2d(Chan.whole(x), packed, b, n, h, w, cout, 1, 1, 0, 0,
                                         "ReLU", out=Chan.whole(out), bk=bk), a.reps)
        wm = wt.view(cout, cin).t().contiguous()
        us_g = timeit(lambda: ops.gemm(x, wm, out=out, bias=b), a.reps)
        fl = 2.0 * n * h * w * cin * cout
        print(f"1x1 {cin:4d}->{cout:4d} (bk {bk}): conv dispatch {us_c:6.1f} us ({fl / us_c / 1e6:6.1f} TF/s)   "
              f"gemm_f32 {us_g:6.1f} us ({fl / us_g / 1e6:6.1f} TF/s)")


if __name__ == "__main__":
    main()
