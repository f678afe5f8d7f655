"""Training step only (BASELINE configs[3] per GPU), for rocprofv3 runs: W warmup + K timed steps.

usage: python tools/train_bench.py [--batch 16] [--steps 3] [--warmup 2] [--iters 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    import bench
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    dev = torch.device("cuda", 0)
    ref = bench.build_refiner(a.iters, dev).train()
    raw = synthetic.make_train_batch(a.batch, a.size, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS, graph=a.graph)
    for _ in range(a.warmup):
        step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step(batch)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"ms_per_step": round(el / a.steps * 1e3, 3),
                      "iters_per_s": round(a.batch * a.iters * a.steps / el, 2),
                      "loss": float(out["loss"].detach())}))


if __name__ == "__main__":
    main()
