"""In-process A/B timing of decoder variants (toggles on one SCFlowDecoder), interleaved.

usage: python tools/ab_bench.py [--batch 16] [--rounds 5] [--steps 10] attr=v1,v2 [attr=...]
e.g.   python tools/ab_bench.py split_pose_conv1=1,0 hoist_context=1,0
       python tools/ab_bench.py env:SCFLOW_WINO4_DEPTH=0,1   (switches read per launch)
Every combination is timed `rounds` times in round-robin order; prints median ms/forward.
"""
import argparse
import itertools
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("toggles", nargs="*")
    a = ap.parse_args()
    from scflow_amd import MODELS, synthetic
    dev = torch.device("cuda")
    feat = (a.size // 8, a.size // 8) if a.size != 256 else None
    dec = MODELS.build(bench.decoder_cfg(a.iters, feat))
    synthetic.fill_module_(dec)
    dec = dec.to(dev).eval()
    inp = bench.make_inputs(a.batch, a.size, seed=0, device=dev)
    names, values = [], []
    import importlib

    def target(k):  # "attr" → the decoder; "pkg.module.Class.attr" → that class/module
        if "." not in k:
            return dec, k
        path, attr = k.rsplit(".", 1)
        mod, _, cls = path.rpartition(".")
        return getattr(importlib.import_module(mod), cls), attr

    for t in a.toggles:
        k, v = t.split("=")
        names.append(k)
        values.append([int(x) if x.lstrip("-").isdigit() else x for x in v.split(",")])
    combos = list(itertools.product(*values)) if names else [()]
    res = {c: [] for c in combos}

    def apply(c):
        for k, v in zip(names, c):
            if k.startswith("env:"):
                os.environ[k[4:]] = str(v)
                from scflow_amd._lib import reload_switches
                reload_switches()  # launch-time switches are cached by the library
                continue
            obj, attr = target(k)
            setattr(obj, attr, v)
    for c in combos:  # warm every variant (packing, allocator)
        apply(c)
        dec(**inp, invalid_flow_num=0.0)
    for _ in range(a.rounds):
        for c in combos:
            apply(c)
            dec(**inp, invalid_flow_num=0.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                dec(**inp, invalid_flow_num=0.0)
            torch.cuda.synchronize()
            res[c].append((time.perf_counter() - t0) / a.steps * 1e3)
    for c in combos:
        med = statistics.median(res[c])
        print(" ".join(f"{k}={v}" for k, v in zip(names, c)) or "default",
              f"median {med:.3f} ms/fwd  {a.batch * a.iters / med * 1e3:.0f} iters/s  "
              f"runs {[round(x, 3) for x in res[c]]}", flush=True)


if __name__ == "__main__":
    main()
