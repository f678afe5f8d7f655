"""Phase profile of the F(2×2,3×3) Winograd conv from its per-workgroup real-time-clock stamps
(scflow_debug_conv_stamps): prologue / main loop / epilogue per workgroup and how many workgroups
are alive over the launch, for the decoder's shapes at B=16, 32×32 (XHead hidden 128→512,
corr_net.1 256→192, out_net 256→126).

    python tools/dbg/wino_stamps.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(cin, cout, n=16, h=32, name=""):
    from scflow_amd import _lib, ops
    from scflow_amd.modules import ConvRunner
    g = torch.Generator().manual_seed(3)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1).cuda()
    x = torch.randn(n * h * h, cin, generator=g).cuda()
    y = torch.empty(n * h * h, cout, device="cuda")
    r = ConvRunner([conv], "ReLU")
    for _ in range(5):
        r.run(ops.Chan.whole(x), ops.Chan.whole(y), n, h, h)
    torch.cuda.synchronize()
    nb = 64 if cout >= 128 else 32  # 32·NBW output channels per workgroup (an upper bound)
    nwg = n * h * h // 128 * (-(-cout // 32))
    st = torch.zeros(nwg * 4, dtype=torch.int64, device="cuda")
    lib = _lib.load()
    lib.scflow_debug_conv_stamps(st.data_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r.run(ops.Chan.whole(x), ops.Chan.whole(y), n, h, h)
    e1.record()
    torch.cuda.synchronize()
    lib.scflow_debug_conv_stamps(None)
    s = st.view(nwg, 4).cpu().double()
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    s = (s - t0) * 0.01
    span = float(s[:, 3].max())
    d = s[:, 1:] - s[:, :-1]
    life = s[:, 3] - s[:, 0]
    print(f"{name} {cin}->{cout}: {len(s)} WGs, event {e0.elapsed_time(e1) * 1e3:.1f} us, span {span:.1f} us, "
          f"WG lifetime mean {life.mean():.1f} us; prologue {d[:, 0].mean():.2f}, main {d[:, 1].mean():.2f}, "
          f"epilogue {d[:, 2].mean():.2f} us (means); starts {s[:, 0].min():.1f}..{s[:, 0].max():.1f}")
    ts = np.linspace(0, span, 16)
    alive = [int(((s[:, 0] <= t) & (s[:, 3] >= t)).sum()) for t in ts]
    mains = [int(((s[:, 1] <= t) & (s[:, 2] >= t)).sum()) for t in ts]
    print("   alive:", alive)
    print("   in main loop:", mains)


if __name__ == "__main__":
    run(128, 512, name="heads")
    run(256, 192, name="corr_net.1")
    run(256, 126, name="out_net")
    run(128, 64, name="delta-flow enc")
