"""Phase split of the F(2×2,3×3) Winograd conv per workgroup (scflow_debug_conv_stamps: start,
prologue done, main loop done, epilogue done on the 100 MHz real-time clock) for the decoder's
shapes at B=16, 32×32: where a launch's time goes (dispatch spread, prologue, K loop, epilogue).

    python tools/dbg/wino_phases.py [--batch 16]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--only", default=None, help="shapes whose name contains this")
    ap.add_argument("--no-stamps", action="store_true", help="timing only (for counter runs)")
    a = ap.parse_args()
    from scflow_amd import _lib
    from scflow_amd.modules import ConvRunner
    from scflow_amd.ops import Chan
    lib = _lib.load()
    lib.scflow_debug_conv_stamps.argtypes = [ctypes.c_void_p]
    n, h, w = a.batch, 32, 32
    M = n * h * w
    shapes = [("heads 128->512", 128, 512), ("corr_net.1 256->192", 256, 192),
              ("out_net 256->126", 256, 126), ("flow_net.1 128->64", 128, 64),
              ("mask_enc.1 64->32", 64, 32), ("corr_net.0 1x1 324->256", 324, 256)]
    for name, cin, cout in shapes:
        if a.only and a.only not in name:
            continue
        k = 1 if "1x1" in name else 3
        conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2).cuda()
        x = torch.randn(M, cin, device="cuda")
        out = torch.empty(M, cout, device="cuda")
        r = ConvRunner([conv], None)

        def run():
            r.run(Chan.whole(x), Chan.whole(out), n, h, w)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(20):
            run()
        ev1.record()
        torch.cuda.synchronize()
        us = ev0.elapsed_time(ev1) * 1e3 / 20
        if a.no_stamps or k == 1:  # (stamps: the Winograd kernel only)
            print(f"{name:22s} {us:6.1f} us/launch", flush=True)
            continue
        st = torch.zeros(65536 * 4, dtype=torch.int64, device="cuda")
        lib.scflow_debug_conv_stamps(ctypes.c_void_p(st.data_ptr()))
        run()
        torch.cuda.synchronize()
        lib.scflow_debug_conv_stamps(None)
        s = st.view(-1, 4).cpu().numpy()
        s = s[s[:, 0] != 0].astype(np.float64) * 0.01  # 100 MHz ticks → µs
        t0 = s[:, 0].min()
        pro, main, epi = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
        print(f"{name:22s} {us:6.1f} us/launch  wgs {len(s):5d}  start spread {s[:, 0].max() - t0:5.2f}  "
              f"prologue {pro.mean():5.2f}  main {main.mean():6.2f}  epilogue {epi.mean():5.2f}  "
              f"last end {s[:, 3].max() - t0:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
