"""The pyramid window lookup alone (a2, scflow_corr_lookup_tiled) at a BASELINE config, HIP-event
timed over many launches, against bench.py's algorithmic byte count (window regions + output).

usage: python tools/lookup_bench.py [--batch 32] [--size 512] [--reps 50] [--check]
  --check: also compare with the row-major lookup (scflow_corr_lookup) on the untiled pyramid
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="per-workgroup phase stamps of one launch")
    ap.add_argument("--flow-scale", type=float, default=6.0, help="flow = randn · scale (px)")
    a = ap.parse_args()
    from scflow_amd import ops
    from scflow_amd.ops import Chan
    dev = torch.device("cuda", 0)
    n, h = a.batch, a.size // 8
    w, L, r, c = h, 4, 4, 256
    g = torch.Generator(device=dev).manual_seed(5)
    f1 = torch.randn(n, c, h, w, device=dev, generator=g)
    f2 = torch.randn(n, c, h, w, device=dev, generator=g)
    pyr = ops.corr_pyramid_tiled(f1, f2, L)
    flow = (torch.randn(n, h, w, 2, device=dev, generator=g) * a.flow_scale).contiguous()
    K = L * (2 * r + 1) ** 2
    out = torch.empty(n * h * w, K, device=dev)
    ch = Chan.whole(out)

    def run():
        ops.corr_lookup(pyr, flow, n, h, w, L, r, out=ch, flow_layout="nhwc", tiled=True)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    P = h * w
    nbytes = n * (4 * P * sum(min(100, P // 4 ** l) for l in range(L)) + 4 * P * K)
    print(f"lookup n={n} {h}x{w} L={L} r={r}: {ms * 1e3:.1f} us/launch, "
          f"{nbytes / 1e6:.1f} MB algorithmic, {nbytes / ms / 1e6:.0f} GB/s "
          f"({nbytes / ms / 1e6 / 8000:.3f} of 8 TB/s)")
    if a.stamps:
        from scflow_amd import _lib
        lib = _lib.load()
        nwg = -(-n * h * w // 16)
        st = torch.zeros(nwg * 6, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        lib.scflow_debug_lookup_stamps(st.data_ptr())
        run()
        torch.cuda.synchronize()
        lib.scflow_debug_lookup_stamps(None)
        v = st.view(-1, 6).double().cpu() / 100.0  # 100 MHz ticks → µs
        t0 = v[:, 0].min()
        names = ("coords", "loads", "lds", "samples", "stores")
        ph = " ".join(f"{nm} {(v[:, i + 1] - v[:, i]).median().item():5.2f}" for i, nm in enumerate(names))
        print(f"  {nwg} WGs span {(v[:, 5].max() - t0).item():7.2f} us, WG median {(v[:, 5] - v[:, 0]).median().item():5.2f} us; "
              f"phase medians (us): {ph}")
    if a.check:
        ref = torch.empty_like(out)
        flat = torch.cat([v.reshape(-1) for v in ops.untile_pyramid(pyr, n, h, w, L)])
        ops.corr_lookup(flat, flow, n, h, w, L, r, out=Chan.whole(ref), flow_layout="nhwc")
        torch.cuda.synchronize()
        err = (out - ref).abs().max().item()
        print(f"max |tiled - row-major| = {err:.3e}")
        assert err == 0.0


if __name__ == "__main__":
    main()
