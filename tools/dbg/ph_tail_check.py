"""GPU check of the fused pose-head tail (scflow_ph_tail) against the unfused launches, printing
the sync words' diagnostics (give-up ticket / counter / value / target / phase, per-workgroup
last ticket) when a dependency wait gives up.

    python tools/dbg/ph_tail_check.py [n] [feat] [reps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from scflow_amd import ops, synthetic
    from scflow_amd.modules import MultiClassPoseHead
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    feat = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    head = MultiClassPoseHead(21, 224, "Basic", dict(type="GN", num_groups=32), dict(type="ReLU"),
                              feat_size=(feat, feat), rotation_mode="ortho6d")
    synthetic.fill_module_(head, seed=7)
    head = head.cuda()
    g = torch.Generator().manual_seed(8)
    x = torch.relu(torch.randn(n, 224, feat, feat, generator=g))
    label = torch.randint(0, 21, (n,), generator=g).cuda()
    hbuf = torch.zeros(n * feat * feat, 384, device="cuda")
    fbuf = torch.zeros(n * feat * feat, 96, device="cuda")
    ops.nchw_into(x[:, :128].contiguous().cuda(), ops.Chan(hbuf, 0, 128))
    ops.nchw_into(x[:, 128:].contiguous().cuda(), ops.Chan.whole(fbuf))
    src0, src1 = ops.Chan(hbuf, 0, 128), ops.Chan.whole(fbuf)
    r, tt = head.forward_hip(src0, src1, n, feat, feat, label)
    torch.cuda.synchronize()
    print("tail_supported", head.tail_supported(src0, src1, n, feat, feat), flush=True)
    ctx = head.tail_conv1(src0, src1, n, feat, feat)
    r3 = torch.empty(n, 6, device="cuda")
    t3 = torch.empty(n, 3, device="cuda")
    args = head.tail_args(ctx, label, r3, t3)
    print("splits", ctx["tail_ws"]["splits"], flush=True)
    ok = True
    for rep in range(reps):
        t0 = time.perf_counter()
        ops.ph_tail(args, r3)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        s = ctx["tail_ws"]["sync"].cpu()
        nc = 16 + 4 * n
        print(f"rep {rep}: {el * 1e3:.2f} ms  ticket={int(s[0])} err={int(s[2])} "
              f"globals={s[3:7].tolist()} giveup(ticket,ctr,val,target,ph+1)={s[9:14].tolist()}",
              flush=True)
        print("  per-sample counters", s[16:nc].view(4, n).tolist(), flush=True)
        if int(s[2]):
            ok = False
            last = s[nc:nc + 512]
            print("  per-WG last ticket (first 64):", last[:64].tolist(), flush=True)
        dr = (r3 - r).abs().max().item()
        dtt = (t3 - tt).abs().max().item()
        print(f"  |drot - unfused| {dr:.3e}  |dt - unfused| {dtt:.3e}", flush=True)
    # per-phase profile from the real-time-clock stamps (100 MHz)
    c = 128
    hs = [feat // 2, feat // 4, feat // 8]
    sp = ctx["tail_ws"]["splits"]
    items = [n * c // 32, -(-n * hs[1] ** 2 // 32) * (c // 32) * sp[0], n * c // 32,
             -(-n * hs[2] ** 2 // 32) * (c // 32) * sp[1], n * c // 32, 64 * 4, 16 * 4, 1]
    total = sum(items)
    stamps = torch.zeros(4 * total, dtype=torch.int64, device="cuda")
    args.stamps = stamps.data_ptr()
    ops.ph_tail(args, r3)
    torch.cuda.synchronize()
    st = stamps.view(total, 4).cpu().double()
    t0 = st[:, 0].min()
    st = (st - t0) * 0.01  # us
    names = ["gn1", "conv2", "gn2", "conv3", "gn3", "fc1", "fc2", "heads"]
    o = 0
    for nm, k in zip(names, items):
        x = st[o:o + k]
        o += k
        print(f"  {nm:6s} items {k:4d}  start {x[:, 0].min():7.2f}..{x[:, 0].max():7.2f}  "
              f"deps-met max {x[:, 1].max():7.2f}  end {x[:, 3].min():7.2f}..{x[:, 3].max():7.2f}  "
              f"avg wait {(x[:, 1] - x[:, 0]).mean():6.2f}  body {(x[:, 2] - x[:, 1]).mean():6.2f}  "
              f"publish {(x[:, 3] - x[:, 2]).mean():6.2f} us", flush=True)
    args.stamps = None
    # timing (events) fused vs unfused
    for name, fn in (("unfused", lambda: head.forward_hip(src0, src1, n, feat, feat, label)),
                     ("fused", lambda: (head.tail_conv1(src0, src1, n, feat, feat),
                                        ops.ph_tail(args, r3)))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per pose head", flush=True)
    print("OK" if ok else "FAILED", flush=True)


if __name__ == "__main__":
    main()
