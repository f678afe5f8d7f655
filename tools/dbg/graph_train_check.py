"""TrainStep(graph=True) vs eager over many steps from the same initial weights: per-step loss
and gradient norm (a replayed graph must follow the eager trajectory's magnitude; step-for-step
equality is not expected with lr > 0 — AdamW amplifies last-bit gradient differences).

usage: python tools/dbg/graph_train_check.py [--steps 16] [--lr 4e-4] [--batch 4]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--lr", type=float, default=4e-4)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--nosync", action="store_true", help="read the losses only after the last step")
    a = ap.parse_args()
    import bench
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    dev = torch.device("cuda", 0)
    ref0 = bench.build_refiner(8, dev).train()
    raw = synthetic.make_train_batch(a.batch, 256, seed=2000)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    for graph in (False, True):
        ref = copy.deepcopy(ref0)
        step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS, lr=a.lr, graph=graph)
        rows = []
        outs = []
        for i in range(a.steps):
            o = step(batch)
            if a.nosync:
                outs.append((o["loss"], o["grad_norm"]))
            else:
                rows.append((float(o["loss"]), float(o["grad_norm"])))
        torch.cuda.synchronize()
        rows += [(float(l), float(g)) for l, g in outs]
        print(("graph" if graph else "eager"), " ".join(f"{l:.4g}/{g:.3g}" for l, g in rows), flush=True)


if __name__ == "__main__":
    main()
