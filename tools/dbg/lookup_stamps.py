"""Phase profile of the pyramid lookup kernel from its real-time-clock stamps
(scflow_debug_lookup_stamps): per workgroup start / coordinates / window loads issued / windows in
LDS / samples / stored, at configs[1] (B=16, 32²) and configs[4] (B=32, 64²).

    python tools/dbg/lookup_stamps.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(n, h, tiled=True):
    from scflow_amd import _lib, ops
    g = torch.Generator().manual_seed(1)
    f1 = torch.randn(n, 256, h, h, generator=g).cuda()
    f2 = torch.randn(n, 256, h, h, generator=g).cuda()
    pyr = ops.corr_pyramid_tiled(f1, f2, 4) if tiled else ops.corr_pyramid(f1, f2, 4)[0]
    flow = ((torch.rand(n * h * h, 2, generator=g) - 0.5) * 8).cuda()
    out = torch.empty(n * h * h, 324, device="cuda")
    for _ in range(3):
        ops.corr_lookup(pyr, flow, n, h, h, 4, 4, out=ops.Chan.whole(out), flow_layout="nhwc", tiled=tiled)
    nwg = (n * h * h + 15) // 16
    st = torch.zeros(nwg * 6, dtype=torch.int64, device="cuda")
    lib = _lib.load()
    torch.cuda.synchronize()
    lib.scflow_debug_lookup_stamps(st.data_ptr())
    ops.corr_lookup(pyr, flow, n, h, h, 4, 4, out=ops.Chan.whole(out), flow_layout="nhwc", tiled=tiled)
    torch.cuda.synchronize()
    lib.scflow_debug_lookup_stamps(None)
    s = st.view(nwg, 6).cpu().double()
    t0 = s[:, 0].min()
    s = (s - t0) * 0.01  # µs
    span = s[:, 5].max()
    d = s[:, 1:] - s[:, :-1]
    names = ["coords", "issue loads", "loads->LDS", "sample", "store"]
    print(f"B={n} {h}x{h} tiled={tiled}: {nwg} WGs, span {span:.1f} us, WG lifetime mean "
          f"{(s[:, 5] - s[:, 0]).mean():.1f} us, starts {s[:, 0].min():.1f}..{s[:, 0].max():.1f} us")
    for k, nm in enumerate(names):
        print(f"   {nm:12s} mean {d[:, k].mean():6.2f}  p50 {d[:, k].median():6.2f}  max {d[:, k].max():6.2f} us")
    # concurrency: how many WGs were alive over time
    import numpy as np
    ts = np.linspace(0, float(span), 20)
    alive = [int(((s[:, 0] <= t) & (s[:, 5] >= t)).sum()) for t in ts]
    print("   alive WGs over the span:", alive)


if __name__ == "__main__":
    run(16, 32)
    run(32, 64)
    run(32, 64, tiled=False)
