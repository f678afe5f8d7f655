"""Time every convolution shape of the decoder in isolation (B pairs, 32×32 features).

usage: python tools/conv_bench.py [--batch 16] [--reps 20]
Prints one line per shape: µs per launch and achieved TFLOP/s (algorithmic FLOPs, fp32).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scflow_amd import ops  # noqa: E402
from scflow_amd._lib import EPI_GRU_Q, EPI_GRU_ZR  # noqa: E402
from scflow_amd.modules import ConvRunner  # noqa: E402
from scflow_amd.ops import Chan  # noqa: E402

# name, cin0, cin1, cout, k, pad, act, epilogue
SHAPES = [
    ("corr_net.0 1x1 324->256", 324, 0, 256, (1, 1), (0, 0), "ReLU", None),
    ("corr_net.1 3x3 256->192", 256, 0, 192, (3, 3), (1, 1), "ReLU", None),
    ("flow_net.0 7x7 2->128", 2, 0, 128, (7, 7), (3, 3), "ReLU", None),
    ("flow_net.1 3x3 128->64", 128, 0, 64, (3, 3), (1, 1), "ReLU", None),
    ("out_net 3x3 256->126", 192, 64, 126, (3, 3), (1, 1), "ReLU", None),
    ("gru zr 1x5 384->256", 384, 0, 256, (1, 5), (0, 2), "Sigmoid", "zr"),
    ("gru q 1x5 128+256->128", 128, 256, 128, (1, 5), (0, 2), "Tanh", "q"),
    ("gru zr 5x1 384->256", 384, 0, 256, (5, 1), (2, 0), "Sigmoid", "zr"),
    ("gru q 5x1 128+256->128", 128, 256, 128, (5, 1), (2, 0), "Tanh", "q"),
    ("gru zr 1x5 128+128->256 +map", 128, 128, 256, (1, 5), (0, 2), "Sigmoid", "zrm"),
    ("gru q 1x5 128+128->128 +map", 128, 128, 128, (1, 5), (0, 2), "Tanh", "qm"),
    ("gru zr 5x1 128+128->256 +map", 128, 128, 256, (5, 1), (2, 0), "Sigmoid", "zrm"),
    ("gru q 5x1 128+128->128 +map", 128, 128, 128, (5, 1), (2, 0), "Tanh", "qm"),
    ("gru ctx map 1x5 128->384", 128, 0, 384, (1, 5), (0, 2), None, None),
    ("heads 3x3 128->512", 128, 0, 512, (3, 3), (1, 1), "ReLU", None),
    ("flow_pred 3x3 256->2", 256, 0, 2, (3, 3), (1, 1), None, None),
    ("mask_pred 1x1 256->1", 256, 0, 1, (1, 1), (0, 0), "Sigmoid", None),
    ("dflow.1 3x3 128->64", 128, 0, 64, (3, 3), (1, 1), "ReLU", None),
    ("mask_enc.0 3x3 1->64", 1, 0, 64, (3, 3), (1, 1), "ReLU", None),
    ("mask_enc.1 3x3 64->32", 64, 0, 32, (3, 3), (1, 1), "ReLU", None),
]


XCD_REPORT = False


def stamp_report(run):
    """One launch of ``run`` with workgroup stamps: spread of the start times, and the median /
    max of each phase (prologue, main loop, epilogue) over the workgroups, in µs."""
    from scflow_amd import _lib
    lib = _lib.load()
    st = torch.zeros(4 * 8192, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    lib.scflow_debug_conv_stamps(st.data_ptr())
    run()
    torch.cuda.synchronize()
    lib.scflow_debug_conv_stamps(None)
    v = st.view(-1, 4).cpu()
    v = v[v[:, 0] > 0].double() / 100.0  # ticks (10 ns) → µs
    if not len(v):
        print("    (no stamps: not a Winograd F(2x2,3x3) launch)")
        return
    t0 = v[:, 0].min()
    ph = [v[:, 1] - v[:, 0], v[:, 2] - v[:, 1], v[:, 3] - v[:, 2]]
    q = lambda x: f"{x.median().item():6.2f}/{x.max().item():6.2f}"
    print(f"    {len(v)} WGs  start spread {(v[:, 0] - t0).max().item():6.2f} us  span "
          f"{(v[:, 3].max() - t0).item():6.2f} us  prologue {q(ph[0])}  main {q(ph[1])}  "
          f"epilogue {q(ph[2])} (median/max us)", flush=True)
    if XCD_REPORT:  # main loop per XCD (linear block id mod 8) and per dispatch round (id / 256)
        ids = torch.nonzero(st.view(-1, 4)[:, 0].cpu() > 0).flatten()
        mn = ph[1]
        print("    main by XCD  " + "  ".join(f"{x}:{q(mn[ids % 8 == x])}" for x in range(8)), flush=True)
        rounds = sorted(set((ids // 256).tolist()))
        print("    main by round " + "  ".join(f"{r}:{q(mn[ids // 256 == r])}" for r in rounds), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="comma-separated substrings of the shapes to run")
    ap.add_argument("--no-extras", action="store_true", help="skip the pyramid / lookup timings")
    ap.add_argument("--xcd", action="store_true", help="with --stamps: main loop per XCD / round")
    ap.add_argument("--stamps", action="store_true",
                    help="Winograd shapes: per-workgroup phase times of one launch "
                         "(scflow_debug_conv_stamps; s_memrealtime at 100 MHz)")
    a = ap.parse_args()
    global XCD_REPORT
    XCD_REPORT = a.xcd
    n, h, w = a.batch, a.size, a.size
    M = n * h * w
    dev = "cuda"
    res = []
    tot_us = 0.0
    for name, c0, c1, cout, k, pad, act, epi in SHAPES:
        if a.only and not any(t in name for t in a.only.split(",")):
            continue
        conv = torch.nn.Conv2d(c0 + c1, cout, k, padding=pad).to(dev)
        x0 = torch.randn(M, c0, device=dev)
        x1 = torch.randn(M, c1, device=dev) if c1 else None
        r = ConvRunner([conv], act)
        kw = {}
        bmap = torch.randn(M, 768, device=dev) if epi in ("zrm", "qm") else None
        if epi in ("zrm", "qm"):
            kw["bias_map"] = Chan(bmap, 0, 256 if epi == "zrm" else 128)
            epi = epi[:-1]
        if epi == "zr":
            hid = torch.randn(M, 128, device=dev)
            kw.update(epilogue=EPI_GRU_ZR, gate=Chan.whole(torch.empty(M, 128, device=dev)),
                      rh=Chan.whole(torch.empty(M, 128, device=dev)), hid=Chan.whole(hid))
            out = None
        elif epi == "q":
            kw.update(epilogue=EPI_GRU_Q, gate=Chan.whole(torch.rand(M, 128, device=dev)),
                      hid=Chan.whole(torch.randn(M, 128, device=dev)))
            out = None
        else:
            out = Chan.whole(torch.empty(M, cout, device=dev))
        src1 = Chan.whole(x1) if x1 is not None else None

        def run():
            r.run(Chan.whole(x0), out, n, h, w, src1=src1, **kw)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        flops = 2.0 * M * cout * (c0 + c1) * k[0] * k[1]
        tf = flops / us / 1e6
        tot_us += us
        res.append(dict(name=name, us=round(us, 2), tflops=round(tf, 2)))
        print(f"{name:28s} {us:9.2f} us  {tf:7.2f} TFLOP/s", flush=True)
        if a.stamps and k in ((3, 3), (1, 5), (5, 1), (7, 7)):
            stamp_report(run)
    print(f"{'sum (one of each)':28s} {tot_us:9.2f} us")
    if a.no_extras:
        return
    # a1 pyramid + a2 lookup (algorithmic bytes: SURVEY.md §8(d))
    C, P = 256, h * w
    f1 = torch.randn(n, C, h, w, device=dev)
    f2 = torch.randn(n, C, h, w, device=dev)
    flow = (torch.rand(n * P, 2, device=dev) - 0.5) * 8

    def timed(fn, reps):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(reps):
            fn()
        e0.record()
        torch.cuda.synchronize()
        return s0.elapsed_time(e0) * 1e3 / reps

    holder = {}

    def build():
        holder["pyr"], _ = ops.corr_pyramid(f1, f2, 4)

    us = timed(build, a.reps)
    fl = 2.0 * n * P * P * C
    print(f"{'corr pyramid (GEMM+pool)':28s} {us:9.2f} us  {fl / us / 1e6:7.2f} TFLOP/s")
    out = Chan.whole(torch.empty(n * P, 324, device=dev))
    us = timed(lambda: ops.corr_lookup(holder["pyr"], flow, n, h, w, 4, 4, out=out, flow_layout="nhwc"),
               a.reps)
    byts = n * (4 * P * sum(min(100, P // 4 ** l) for l in range(4)) + 4 * P * 324)
    print(f"{'corr lookup r=4':28s} {us:9.2f} us  {byts / us / 1e3:7.2f} GB/s (algorithmic)")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
