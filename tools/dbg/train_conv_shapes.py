"""Per-shape timing of the training step's conv launches (forward / dgrad via the conv dispatch,
weight gradients via ops.conv_wgrad): every call is bracketed with HIP events on its stream,
aggregated by (op, shape) over one step at configs[3] (B=16, 256², 8 iterations), with the
algorithmic fp32 flops and the achieved TFLOP/s of each shape.

    python tools/dbg/train_conv_shapes.py [--batch 16]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    import bench
    from scflow_amd import ops, synthetic
    from scflow_amd.train import functions
    from scflow_amd.train.step import TrainStep

    rec = []
    on = [False]

    def wrap(name, fn, flops):
        def f(*args, **kw):
            if not on[0]:
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # drain, then keep the GPU busy while the host enqueues the call: the events then
            # bracket the call's kernels only, not the host's argument marshalling
            torch.cuda.synchronize()
            torch.cuda._sleep(2_000_000)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            key, fl = flops(*args, **kw)
            rec.append((name, key, fl, e0, e1))
            return r
        return f

    def wg_flops(dy, src0, src1, dw, db, n, h, w, kh, kw, stride, ph, pw, accumulate=False):
        cout, cin = dw.shape[0], dw.shape[1]
        oh, ow = (h + 2 * ph - kh) // stride + 1, (w + 2 * pw - kw) // stride + 1
        return ((n, h, w, cin, cout, kh, kw, stride), 2.0 * n * oh * ow * cout * cin * kh * kw)

    def fw_flops(x0, x1, w, b, stride, pad, act=None, bias_map=None, wkey=None):
        n, h, wd, c0 = x0.shape
        cin = c0 + (0 if x1 is None else x1.shape[-1])
        cout, _, kh, kw = w.shape
        oh, ow = (h + 2 * pad[0] - kh) // stride + 1, (wd + 2 * pad[1] - kw) // stride + 1
        return ((n, h, wd, cin, cout, kh, kw, stride), 2.0 * n * oh * ow * cout * cin * kh * kw)

    def gemm_flops(a_, b_, out=None, alpha=1.0, beta=0.0, bias=None, bias_dim="n"):
        bt = a_.shape[0] if a_.dim() == 3 else 1
        m, k = a_.shape[-2:]
        nn = b_.shape[-1]
        # caller: the innermost frame outside ops.py (which Function's forward / backward)
        import inspect
        fr = inspect.currentframe().f_back.f_back
        tag = f"{os.path.basename(fr.f_code.co_filename)}:{fr.f_lineno}"
        return ((bt, m, nn, k, tag, 0, 0, 0), 2.0 * bt * m * nn * k)

    def wgb_flops(dys, src0s, src1s, dw, db, n, h, w, kh, kw, stride, ph, pw, accumulate=False):
        cout, cin = dw.shape[0], dw.shape[1]
        segs = len(dys)
        return ((segs * n, h, w, cin, cout, kh, kw, stride), 2.0 * segs * n * h * w * cout * cin * kh * kw)

    ops.conv_wgrad = wrap("wgrad", ops.conv_wgrad, wg_flops)
    ops.conv_wgrad_batched = wrap("wgb", ops.conv_wgrad_batched, wgb_flops)
    ops.gemm = wrap("gemm", ops.gemm, gemm_flops)
    functions._conv_forward = wrap("conv", functions._conv_forward, fw_flops)

    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(8, dev).train()
    raw = synthetic.make_train_batch(a.batch, 256, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS)
    for _ in range(3):
        step(batch)
    torch.cuda.synchronize()
    on[0] = True
    step(batch)
    torch.cuda.synchronize()
    on[0] = False
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for name, key, fl, e0, e1 in rec:
        g = agg[(name,) + key]
        g[0] += 1
        g[1] += e0.elapsed_time(e1) * 1e3
        g[2] += fl
    tot = sum(v[1] for v in agg.values())
    print(f"conv + wgrad launches of one step: {len(rec)} calls, {tot / 1e3:.2f} ms (host-timed events)")
    print(" op     n   h   w  cin cout kh kw s | calls   total_us  avg_us  GFLOP/call  TF/s")
    for k, (c, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if k[0] == "gemm":  # (batch, M, N, K, caller)
            print(f" gemm  bt={k[1]} M={k[2]} N={k[3]} K={k[4]} {k[5]} | {c:5d} {us:10.1f} {us / c:7.1f}"
                  f" {fl / c / 1e9:10.3f} {fl / us / 1e6:6.1f}")
            continue
        print(f" {k[0]:5s} {k[1]:3d} {k[2]:3d} {k[3]:3d} {k[4]:4d} {k[5]:4d} {k[6]:2d} {k[7]:2d} {k[8]:1d} |"
              f" {c:5d} {us:10.1f} {us / c:7.1f} {fl / c / 1e9:10.3f} {fl / us / 1e6:6.1f}")


if __name__ == "__main__":
    main()
